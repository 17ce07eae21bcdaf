"""conv5_x-shaped (N=4, 24x78, 512->512 3x3) forward / input-gradient
launches under kernel options (halo 256x256 split-K vs 256x128 vs implicit
GEMM).  Diagnostic only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semanticsegmentation_tensorflow_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
ws = ops.Workspace(dev)
MODES = [("default", {}), ("halo128", {"halo_wide": 0}), ("igemm", {"nt_halo": 0}),
         ("igemm-nt2", {"nt_halo": 0, "nt3": 0})]
RESET = {"halo_wide": 1, "nt_halo": 1, "nt3": 1}


def timeit(fn, reps=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


for (N, H, W, C, K) in [(4, 24, 78, 512, 512), (4, 48, 156, 512, 512), (4, 192, 624, 128, 128)]:
    d = ops.conv_desc(N, H, W, C, K, 3, 3, dtype=ops.BF16)
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    wk = (torch.randn(K, 3, 3, C, device=dev) * 0.02).to(torch.bfloat16)
    y = torch.empty(N, H, W, K, device=dev, dtype=torch.bfloat16)
    gf = 2.0 * N * H * W * 9 * C * K / 1e9
    for name, opts in MODES:
        for k, v in {**RESET, **opts}.items():
            ops.set_option(k, v)
        t = min(timeit(lambda: ops.conv2d_fwd(d, x, wk, y, None, ws)) for _ in range(3))
        print(f"{N}x{H}x{W} {C}->{K} {name:10s} fwd {t * 1e3:7.1f} us {gf / t:7.1f} TF/s {ops.conv_kernel_info(d, 0)[:2]}",
              flush=True)
for k, v in RESET.items():
    ops.set_option(k, v)
