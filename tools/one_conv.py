"""Run one FCN conv op repeatedly (profiling target).
    python tools/one_conv.py LAYER OP VARIANT REPS   (OP: fwd|dgrad|wgrad)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semanticsegmentation_tensorflow_amd import ops  # noqa: E402
from tools.convbench import LAYERS  # noqa: E402

name, op, var, reps = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
N = 4
L = {l[0]: l for l in LAYERS}[name]
_, H, W, C, K, R = L
dev = torch.device("cuda:0")
ws = ops.Workspace(dev)
ops.set_option("igemm_nt_variant", var)
ops.set_option("igemm_tn_variant", var)
d = ops.conv_desc(N, H, W, C, K, R, R, dtype=ops.BF16)
x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
wk = (torch.randn(K, R, R, C, device=dev) * 0.05).to(torch.bfloat16)
wh = (torch.randn(R, R, C, K, device=dev) * 0.05).to(torch.bfloat16)
y = torch.empty(N, d.OH, d.OW, K, device=dev, dtype=torch.bfloat16)
dx = torch.empty_like(x)
dw = torch.empty(R, R, C, K, device=dev)
fn = {"fwd": lambda: ops.conv2d_fwd(d, x, wk, y, ops.epilogue(relu=True), ws),
      "dgrad": lambda: ops.conv2d_bwd_data(d, y, wh, dx, ws),
      "wgrad": lambda: ops.conv2d_bwd_filter(d, x, y, dw, ws)}[op]
for _ in range(reps):
    fn()
torch.cuda.synchronize()
print("done", name, op, var, ops.conv_kernel_info(d, {"fwd": 0, "dgrad": 1, "wgrad": 2}[op]))
