"""Ablations of conv_res64 on conv1_2 (diagnostic; outputs garbage for ablate > 0)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semanticsegmentation_tensorflow_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
ws = ops.Workspace(dev)
d = ops.conv_desc(4, 384, 1248, 64, 64, 3, 3, dtype=ops.BF16)
x = torch.randn(4, 384, 1248, 64, device=dev).to(torch.bfloat16)
wk = (torch.randn(64, 3, 3, 64, device=dev) * 0.05).to(torch.bfloat16)
y = torch.empty_like(x)
names = {0: "full", 1: "no-fetch", 2: "no-MFMA", 3: "no-store", 4: "no-LDS-read"}
res = {a: [] for a in names}
for rnd in range(4):
    for a in names:
        ops.set_option("nt2_ablate", a)
        ops.conv2d_fwd(d, x, wk, y, None, ws)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            ops.conv2d_fwd(d, x, wk, y, None, ws)
        e.record()
        torch.cuda.synchronize()
        res[a].append(s.elapsed_time(e) / 10)
ops.set_option("nt2_ablate", 0)
print("  ".join(f"{names[a]}={min(v) * 1e3:.1f}us" for a, v in res.items()))
