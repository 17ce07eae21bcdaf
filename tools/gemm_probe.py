"""Square bf16 GEMMs through the conv entry point (1x1 filter: M = pixels,
N = K = channels) on random data: how igemm_nt3 compares with the guide's
256^2 8-phase template (~1.32 PF/s at 4096^3, ~1.47 at 8192^3).  Diagnostic."""
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


for n in (4096, 8192):
    d = ops.conv_desc(1, n // 64, 64, n, n, 1, 1, dtype=ops.BF16)
    x = (torch.rand(1, n // 64, 64, n, device=dev) * 2 - 1).to(torch.bfloat16)
    w = (torch.rand(n, 1, 1, n, device=dev) * 2 - 1).to(torch.bfloat16)
    y = torch.empty(1, n // 64, 64, n, device=dev, dtype=torch.bfloat16)
    for opt in ("", "nt4=1", "nt4=1,abl"):
        ops.set_option("nt3", 0 if opt == "nt3=0" else 1)
        ops.set_option("nt4", 1 if opt.startswith("nt4=1") else 0)
        ops.set_option("nt4_abl", 1 if opt.endswith("abl") else 0)
        t = min(timeit(lambda: ops.conv2d_fwd(d, x, w, y, None, ws)) for _ in range(3))
        print(f"{n}^3 {opt or 'nt3':6s} {t * 1e3:8.1f} us {2 * n ** 3 / t / 1e9:7.1f} TF/s "
              f"({ops.conv_kernel_info(d, 0)[0]})", flush=True)
    ops.set_option("nt3", 1)
    ops.set_option("nt4", 0)
    ops.set_option("nt4_abl", 0)
    torch.matmul(x.view(n, n), w.view(n, n).t())
    t = min(timeit(lambda: torch.matmul(x.view(n, n), w.view(n, n).t())) for _ in range(3))
    print(f"{n}^3 torch.matmul (hipBLASLt) {t * 1e3:8.1f} us {2 * n ** 3 / t / 1e9:7.1f} TF/s", flush=True)
