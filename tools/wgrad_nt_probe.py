"""conv6 filter gradient as a dense NT GEMM (im2col'd x and transposed dy,
both k = pixel contiguous) vs the TN kernel: the same M x N x K timed as a
1x1 Conv2D on igemm_nt3.  Diagnostic only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semanticsegmentation_tensorflow_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
ws = ops.Workspace(dev)


def timeit(fn, reps=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


for name, M, N, K in [("conv6", 7 * 7 * 512, 4096, 4 * 12 * 39), ("conv7", 4096, 4096, 4 * 12 * 39)]:
    Kp = ops.round8(K)
    for rows in (1, 2, 4):
        d = ops.conv_desc(rows, 1, M // rows, Kp, N, 1, 1, dtype=ops.BF16)
        x = torch.randn(rows, 1, M // rows, Kp, device=dev).to(torch.bfloat16)
        w = torch.randn(N, 1, 1, Kp, device=dev).to(torch.bfloat16)
        y = torch.empty(rows, 1, M // rows, N, device=dev, dtype=torch.bfloat16)
        t = min(timeit(lambda: ops.conv2d_fwd(d, x, w, y, None, ws)) for _ in range(3))
        gf = 2.0 * M * N * K / 1e9
        print(f"{name} NT-equivalent M={M} N={N} K={Kp}: {t * 1e3:8.1f} us {gf / t:7.1f} TF/s "
              f"{ops.conv_kernel_info(d, 0)}", flush=True)
