"""Which C5 conv -> BN pairs take seg_conv2d_fwd_bn2 on the GPU (plan probe)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import bench
from semanticsegmentation_tensorflow_amd import ops
g = bench.build_train_graph("deeplab", 375, 1242, "f16")
sess = g["sess"]
img = np.zeros((2, g["HP"], g["WP"], 3), np.float32)
lab = np.zeros((2, g["HP"], g["WP"]), np.uint8)
sess.run([g["train_step"], g["loss"]], feed_dict={g["image"]: img, g["labels"]: lab, g["keep"]: 0.8})
(p,) = [q for q in sess.plans.values() if q.train]
prod = {id(n.output): n for n in p.nodes if n.kind == "conv"}
for b in p.nodes:
    if b.kind != "bn":
        continue
    c = prod.get(id(b.inputs[0]))
    if c is None:
        print("bn without conv producer")
        continue
    d = c.desc
    print((d.N, d.H, d.W, d.C, d.K, d.R, d.dil_h), ops.conv_kernel_info(d, ops.OP_FWD)[:2],
          "bn2_ok", ops.conv2d_fwd_bn2_ok(d, getattr(c, "pro", None) is not None),
          "planned", id(c) in p.bn_out2, "folded", id(b) in p.folded)
