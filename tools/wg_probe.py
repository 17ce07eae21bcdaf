"""Filter-gradient probe for the 3x3 FCN layers under kernel options
(SEG_OPTIONS-style overrides), interleaved, min over rounds.  Diagnostic only.
    python tools/wg_probe.py "wgrad_la=1" "wgrad_la=2" ..."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semanticsegmentation_tensorflow_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
ws = ops.Workspace(dev)
LAYERS = [("conv1_2", 384, 1248, 64, 64), ("conv2_2", 192, 624, 128, 128), ("conv3_2", 96, 312, 256, 256),
          ("conv4_2", 48, 156, 512, 512), ("conv5_2", 24, 78, 512, 512)]
CONFIGS = sys.argv[1:] or ["wgrad_la=1", "wgrad_la=2"]


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
    dy = torch.randn(N, H, W, K, device=dev).to(torch.bfloat16)
    dw = torch.empty(3, 3, C, K, device=dev)
    db = torch.empty(K, device=dev) if os.environ.get("PROBE_BIAS") else None
    gf = 2.0 * N * H * W * 9 * C * K / 1e9
    best = {c: 1e9 for c in CONFIGS}
    for _ in range(3):
        for c in CONFIGS:
            apply(c)
            best[c] = min(best[c], timeit(lambda: ops.conv2d_bwd_filter(d, x, dy, dw, ws, dbias=db)))
    print(name, " | ".join(f"{c}: {best[c] * 1e3:6.1f}us {gf / best[c]:6.0f}TF" for c in CONFIGS), flush=True)
