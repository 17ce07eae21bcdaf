"""Filter-gradient kernel probe: conv6 / conv7 / conv_t2-shaped TN GEMMs under
kernel options (tn2 vs tn3, tile order, ablations).  Diagnostic only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semanticsegmentation_tensorflow_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
ws = ops.Workspace(dev)
SHAPES = [("conv6", 12, 39, 512, 4096, 7), ("conv7", 12, 39, 4096, 4096, 1)]
MODES = [("tn2", {"tn3": 0}), ("tn3-nfast", {"tn3": 1, "tn3_mfast": 0}), ("tn3-mfast", {"tn3": 1, "tn3_mfast": 1}),
         ("abl-noDMA", {"tn3": 1, "tn3_abl": 1}), ("abl-noMFMA", {"tn3": 1, "tn3_abl": 2}),
         ("abl-noEpi", {"tn3": 1, "tn3_abl": 3}),
         ("tn3-unstag", {"tn3": 1, "tn3_stag": 0}), ("unstag-noDMA", {"tn3": 1, "tn3_stag": 0, "tn3_abl": 1}),
         ("unstag-noEpi", {"tn3": 1, "tn3_stag": 0, "tn3_abl": 3})]


def timeit(fn, reps=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


if len(sys.argv) > 1:   # python tools/tn_probe.py SHAPE MODE  (one config, for PMC passes)
    SHAPES = [sh for sh in SHAPES if sh[0] == sys.argv[1]]
    MODES = [m for m in MODES if m[0] == sys.argv[2]]
for name, H, W, C, K, R in SHAPES:
    N = 4
    d = ops.conv_desc(N, H, W, C, K, R, R, dtype=ops.BF16)
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    dy = torch.randn(N, d.OH, d.OW, K, device=dev).to(torch.bfloat16)
    dw = torch.empty(R, R, C, K, device=dev)
    gf = 2.0 * N * H * W * R * R * C * K / 1e9
    for mname, opts in MODES:
        for k, v in opts.items():
            ops.set_option(k, v)
        t = min(timeit(lambda: ops.conv2d_bwd_filter(d, x, dy, dw, ws)) for _ in range(3))
        print(f"{name:6s} {mname:12s} {t * 1e3:8.1f} us  {gf / t:8.1f} TF/s  {ops.conv_kernel_info(d, 2)[0]}")
        ops.set_option("tn3_abl", 0)
        ops.set_option("tn3_stag", 1)
        ops.set_option("tn3_mfast", 1)
        ops.set_option("tn3", 1)
