"""Time one layer's fwd / dgrad / wgrad (bf16) with HIP events, min over rounds."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semanticsegmentation_tensorflow_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--opt", action="append", default=[], help="name=value seg_set_option before timing")
args = ap.parse_args()
for o in args.opt:
    k, v = o.split("=")
    ops.set_option(k, int(v))
dev = torch.device("cuda:0")
ws = ops.Workspace(dev)
LAYERS = [("conv1_1", 384, 1248, 3, 64, 3), ("conv1_2", 384, 1248, 64, 64, 3), ("conv2_2", 192, 624, 128, 128, 3),
          ("conv3_2", 96, 312, 256, 256, 3), ("conv4_2", 48, 156, 512, 512, 3), ("conv5_2", 24, 78, 512, 512, 3),
          ("conv6", 12, 39, 512, 4096, 7), ("conv7", 12, 39, 4096, 4096, 1)]


def timeit(fn, reps=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / reps)
    return best


for (name, H, W, C, K, R) in LAYERS:
    N = 4
    d = ops.conv_desc(N, H, W, C, K, R, R, dtype=ops.BF16)
    Cp, Kp = ops.round8(C), ops.round8(K)
    x = torch.randn(N, H, W, Cp, device=dev).to(torch.bfloat16)
    dy = torch.randn(N, H, W, Kp, device=dev).to(torch.bfloat16)
    wk = (torch.randn(Kp, R, R, Cp, device=dev) * 0.05).to(torch.bfloat16)
    wh = (torch.randn(R, R, Cp, Kp, device=dev) * 0.05).to(torch.bfloat16)
    y = torch.empty(N, H, W, Kp, device=dev, dtype=torch.bfloat16)
    dx = torch.empty_like(x)
    dw = torch.empty(R, R, C, K, device=dev, dtype=torch.float32)
    db = torch.empty(K, device=dev, dtype=torch.float32)
    out = []
    for op, fn in ((0, lambda: ops.conv2d_fwd(d, x, wk, y, None, ws)),
                   (1, lambda: ops.conv2d_bwd_data(d, dy, wh, dx, ws)),
                   (2, lambda: ops.conv2d_bwd_filter(d, x, dy, dw, ws, None, db))):
        if op == 1 and name == "conv1_1":
            continue
        name_k, sp, flops = ops.conv_kernel_info(d, op)
        t = timeit(fn)
        out.append(f"{['fwd', 'dgrad', 'wgrad'][op]}={t * 1e3:.1f}us({flops / t / 1e9:.0f}TF,{name_k},sp{sp})")
    print(name, "  ".join(out), flush=True)
