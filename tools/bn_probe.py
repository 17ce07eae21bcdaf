"""BN+ReLU forward / backward bandwidth at FC-DenseNet block-1 shapes.  Diagnostic."""
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


for (N, H, W, C) in ((8, 384, 1248, 48), (8, 384, 1248, 96), (8, 384, 1248, 64), (8, 192, 624, 208)):
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    y = torch.empty_like(x)
    dx = torch.empty_like(x)
    g = torch.rand(C, device=dev) + 0.5
    b = torch.rand(C, device=dev)
    dg = torch.zeros(C, device=dev)
    db = torch.zeros(C, device=dev)
    t = timeit(lambda: ops.bn_relu_fwd(x, y, g, b, C))
    byt = x.numel() * 2 * 2
    print(f"fwd {N}x{H}x{W}x{C}: {t * 1e3:7.1f} us {byt / t / 1e9:6.2f} TB/s", flush=True)
    t = timeit(lambda: ops.bn_relu_bwd(x, y, y, dx, g, dg, db, C, True, 1e-3, ws))
    byt = x.numel() * 2 * 4
    print(f"bwd {N}x{H}x{W}x{C}: {t * 1e3:7.1f} us {byt / t / 1e9:6.2f} TB/s", flush=True)
    t = timeit(lambda: y.copy_(x))
    print(f"copy {N}x{H}x{W}x{C}: {t * 1e3:7.1f} us {x.numel() * 4 / t / 1e9:6.2f} TB/s", flush=True)
