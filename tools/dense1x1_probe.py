"""FC-DenseNet bottleneck 1x1 convs at block-1 size (8 x 384 x 1248): the
BN+ReLU-prologue forward (C -> 64) and the input gradient through the BN
backward (64 -> C, accumulating into the concat gradient), in TB/s of
algorithmic bytes.  Diagnostic only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semanticsegmentation_tensorflow_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
ws = ops.Workspace(dev)
for kv in filter(None, os.environ.get("PROBE_OPTS", "").split(",")):
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


N, H, W, K = 8, 384, 1248, 64
P = N * H * W
for C in (48, 112, 208):
    d = ops.conv_desc(N, H, W, C, K, 1, 1, dtype=ops.BF16)
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    y = torch.empty(N, H, W, K, device=dev, dtype=torch.bfloat16)
    g = torch.rand(C, device=dev) + 0.5
    b = torch.rand(C, device=dev) - 0.5
    wk = (torch.randn(K, 1, 1, C, device=dev) * 0.1).to(torch.bfloat16)
    wh = (torch.randn(1, 1, C, K, device=dev) * 0.1).to(torch.bfloat16)
    pro = ops.prologue(g, b)
    kp = float(os.environ.get("PROBE_KP", "0.2"))
    epi = ops.epilogue(keep_prob=kp, seed=7)
    t = min(timeit(lambda: ops.conv2d_fwd_pro(d, x, pro, wk, y, epi, ws)) for _ in range(3))
    byt = P * (C + K) * 2
    t2 = min(timeit(lambda: ops.conv2d_fwd(d, x, wk, y, epi, ws)) for _ in range(3))
    print(f"fwd_plain C={C:3d}: {t2 * 1e3:7.1f} us {byt / t2 / 1e9:6.2f} TB/s  {ops.conv_kernel_info(d, ops.OP_FWD)[0]}",
          flush=True)
    print(f"fwd_pro C={C:3d}: {t * 1e3:7.1f} us {byt / t / 1e9:6.2f} TB/s  {ops.conv_kernel_info(d, ops.OP_FWD_PRO)[0]}",
          flush=True)
    dy = torch.randn(N, H, W, K, device=dev).to(torch.bfloat16)
    dx = torch.zeros(N, H, W, C, device=dev, dtype=torch.bfloat16)
    dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    t = min(timeit(lambda: ops.conv2d_bwd_data_bn(d, dy, wh, x, g, b, dx, dg, db, accumulate=True, ws=ws))
            for _ in range(3))
    byt = P * (K + 3 * C) * 2
    print(f"dgrad_bn C={C:3d}: {t * 1e3:7.1f} us {byt / t / 1e9:6.2f} TB/s  "
          f"{ops.conv_kernel_info(d, ops.OP_BWD_DATA_BN)[0]}", flush=True)
    t = min(timeit(lambda: dx.copy_(x)) for _ in range(3))
    print(f"copy     C={C:3d}: {t * 1e3:7.1f} us {P * C * 4 / t / 1e9:6.2f} TB/s", flush=True)
