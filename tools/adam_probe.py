"""Fused filter-gradient + TF1 Adam probe (conv6 / conv7 shapes): epilogue
ablations vs the plain gradient GEMM and a device copy.  Diagnostic only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semanticsegmentation_tensorflow_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
for kv in filter(None, os.environ.get("PROBE_OPTS", "").split(",")):   # e.g. PROBE_OPTS=tn3_mfast=1
    k, v = kv.split("=")
    ops.set_option(k, int(v))
ws = ops.Workspace(dev)
SHAPES = [("conv6", 12, 39, 512, 4096, 7), ("conv7", 12, 39, 4096, 4096, 1)]
HALF = [int(h) for h in os.environ.get("PROBE_HALF", "1").split(",")]
STAG = [int(h) for h in os.environ.get("PROBE_STAGGER", "0").split(",")]
WSTAG = [int(h) for h in os.environ.get("PROBE_WSTAG", "1").split(",")]
ABL = [0, 1, 2, 3, 4, 8, 12, 16]
ABL = [int(a) for a in os.environ.get("PROBE_ABL", ",".join(map(str, ABL))).split(",")]


def timeit(fn, reps=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


for name, H, W, C, K, R in SHAPES:
    N = 4
    d = ops.conv_desc(N, H, W, C, K, R, R, dtype=ops.BF16)
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    dy = torch.randn(N, d.OH, d.OW, K, device=dev).to(torch.bfloat16)
    dw = torch.empty(R, R, C, K, device=dev)
    p, m, v = (torch.rand(R * R * C * K, device=dev) * 1e-3 for _ in range(3))
    cp, kp = ops.round8(C), ops.round8(K)
    rows = torch.zeros(ops.packed_shape(R, R, C, K, ops.PACK_HWIO), dtype=torch.bfloat16, device=dev)
    tr = torch.zeros(ops.packed_shape(R, R, C, K, ops.PACK_KRSC), dtype=torch.bfloat16, device=dev)
    n = p.numel()
    gf = 2.0 * N * H * W * R * R * C * K / 1e9
    for h, ws_ in [(h, w_) for h in HALF for w_ in WSTAG]:
        ops.set_option("tn3_half", h)
        ops.set_option("tn3_stag", ws_)
        t = min(timeit(lambda: ops.conv2d_bwd_filter(d, x, dy, dw, ws)) for _ in range(3))
        print(f"{name} half={h} wstag={ws_} grad-only  {t * 1e3:8.1f} us {gf / t:7.1f} TF/s", flush=True)
        for a in ABL:
            for sg in STAG:
                ops.set_option("tn3_adam_abl", a)
                ops.set_option("tn3_stagger_us", sg)
                t = min(timeit(lambda: ops.conv2d_bwd_filter_adam(d, x, dy, p, m, v, 1e-4, 3, rows=(rows, cp, kp),
                                                                  tr=(tr, cp, kp), ws=ws)) for _ in range(3))
                print(f"{name} half={h} wstag={ws_} adam abl={a:2d} stagger={sg:3d}us {t * 1e3:8.1f} us "
                      f"({28 * n / t / 1e9:6.2f} TB/s at 28 B/param)", flush=True)
        ops.set_option("tn3_stagger_us", 0)
    ops.set_option("tn3_adam_abl", 0)
    ops.set_option("tn3_stag", 1)
    big = torch.empty(n * 6, device=dev)
    t = min(timeit(lambda: big[: n * 3].copy_(big[n * 3:])) for _ in range(3))
    print(f"{name} copy 12B/param {t * 1e3:8.1f} us ({24 * n / t / 1e9:6.2f} TB/s)", flush=True)
