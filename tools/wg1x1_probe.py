"""1x1 filter-gradient probe (FC-DenseNet bottleneck shapes: few channels x
millions of pixels): split-K fill / cap and tn2-for-small-M sweeps.
Diagnostic only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semanticsegmentation_tensorflow_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
ws = ops.Workspace(dev)
SHAPES = [(384, 1248, 48, 64), (384, 1248, 96, 64), (384, 1248, 128, 64), (384, 1248, 256, 2),
          (192, 624, 160, 80), (96, 312, 192, 64)]
MODES = [("base", {}), ("fill4", {"tn_fill": 4, "tn_split_cap": 1024}),
         ("fill8", {"tn_fill": 8, "tn_split_cap": 2048}),
         ("fill8-smallm", {"tn_fill": 8, "tn_split_cap": 2048, "tn2_smallm": 1}),
         ("fill16-smallm", {"tn_fill": 16, "tn_split_cap": 4096, "tn2_smallm": 1})]
DEFAULTS = {"tn_fill": 2, "tn_split_cap": 256, "tn2_smallm": 0}


def timeit(fn, reps=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


for H, W, C, K in SHAPES:
    N = 8
    d = ops.conv_desc(N, H, W, C, K, 1, 1, dtype=ops.BF16)
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    dy = torch.randn(N, H, W, ops.round8(K), device=dev).to(torch.bfloat16)
    dw = torch.empty(1, 1, C, K, device=dev)
    gb = (x.numel() + dy.numel()) * 2 / 1e9
    ref = None
    for mname, opts in MODES:
        for k, v in {**DEFAULTS, **opts}.items():
            ops.set_option(k, v)
        t = min(timeit(lambda: ops.conv2d_bwd_filter(d, x, dy, dw, ws)) for _ in range(3))
        if ref is None:
            ref = dw.clone()
        err = float((dw - ref).abs().max() / ref.abs().max())
        info = ops.conv_kernel_info(d, 2)
        print(f"{N}x{H}x{W} C={C:3d} K={K:3d} {mname:14s} {t * 1e3:8.1f} us {gb / t * 1e3:7.0f} GB/s "
              f"{info}  err={err:.1e}", flush=True)
for k, v in DEFAULTS.items():
    ops.set_option(k, v)

# folded BatchNorm + ReLU prologue vs the separate bn_relu_fwd pass
for H, W, C, K in SHAPES[:3] + SHAPES[4:]:
    N = 8
    d = ops.conv_desc(N, H, W, C, K, 1, 1, dtype=ops.BF16)
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    xa = torch.empty_like(x)
    w = torch.randn(K, 1, 1, C, device=dev).to(torch.bfloat16)
    y = torch.empty(N, H, W, ops.round8(K), device=dev, dtype=torch.bfloat16)
    dy = torch.randn(N, H, W, ops.round8(K), device=dev).to(torch.bfloat16)
    dw = torch.empty(1, 1, C, K, device=dev)
    g, b = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    pro = ops.prologue(g, b)
    t_bn = min(timeit(lambda: ops.bn_relu_fwd(x, xa, g, b, C)) for _ in range(3))
    t_f = min(timeit(lambda: ops.conv2d_fwd(d, xa, w, y, None, ws)) for _ in range(3))
    t_fp = min(timeit(lambda: ops.conv2d_fwd_pro(d, x, pro, w, y, None, ws)) for _ in range(3))
    t_w = min(timeit(lambda: ops.conv2d_bwd_filter(d, xa, dy, dw, ws)) for _ in range(3))
    t_wp = min(timeit(lambda: ops.conv2d_bwd_filter_pro(d, x, pro, dy, dw, ws)) for _ in range(3))
    print(f"PRO {N}x{H}x{W} C={C:3d} K={K:3d} bn_relu {t_bn * 1e3:7.1f} fwd {t_f * 1e3:7.1f} fwd_pro {t_fp * 1e3:7.1f} "
          f"wgrad {t_w * 1e3:7.1f} wgrad_pro {t_wp * 1e3:7.1f} us", flush=True)
