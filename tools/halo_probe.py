"""conv_halo2 (3x3 fwd / dgrad, N > 128) probe under options, interleaved in
one process, min over rounds.  python tools/halo_probe.py "nt2_ablate=0" ..."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semanticsegmentation_tensorflow_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
ws = ops.Workspace(dev)
LAYERS = [("conv3_2", 96, 312, 256, 256), ("conv4_2", 48, 156, 512, 512)]
CONFIGS = sys.argv[1:] or ["nt2_ablate=0"]


def apply(cfg):
    for kv in filter(None, cfg.split(",")):
        k, v = kv.split("=")
        ops.set_option(k, int(v))


def timeit(fn, reps=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


for name, H, W, C, K in LAYERS:
    N = 4
    d = ops.conv_desc(N, H, W, C, K, 3, 3, dtype=ops.BF16)
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    wk = (torch.randn(K, 3, 3, C, device=dev) * 0.05).to(torch.bfloat16)
    y = torch.empty(N, H, W, K, device=dev, dtype=torch.bfloat16)
    gf = 2.0 * N * H * W * 9 * C * K / 1e9
    best = {c: 1e9 for c in CONFIGS}
    for _ in range(3):
        for c in CONFIGS:
            apply(c)
            best[c] = min(best[c], timeit(lambda: ops.conv2d_fwd(d, x, wk, y, ops.epilogue(relu=True), ws)))
            apply("nt2_ablate=0")
    print(name, " | ".join(f"{c}: {best[c] * 1e3:6.1f}us {gf / best[c]:6.0f}TF" for c in CONFIGS), flush=True)
