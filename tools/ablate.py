"""Kernel timing for the FCN 3x3 layers (diagnostic).

Modes per layer (interleaved rounds in one process, min over rounds):
  nt2       LDS-DMA implicit GEMM
  halo      halo-tiled direct conv (default path)
  nt2-abl1  nt2 without LDS-DMA in the main loop   (garbage output)
  nt2-abl2  nt2 without MFMA                       (garbage output)
  nt2-abl3  nt2 with trivial source addresses      (garbage output)
and the same fwd / dgrad pair for the halo path."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semanticsegmentation_tensorflow_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ablate", action="store_true")
args = ap.parse_args()

dev = torch.device("cuda:0")
ws = ops.Workspace(dev)
LAYERS = [("conv1_2", 384, 1248, 64, 64), ("conv2_2", 192, 624, 128, 128), ("conv3_2", 96, 312, 256, 256),
          ("conv4_2", 48, 156, 512, 512), ("conv5_2", 24, 78, 512, 512)]
MODES = [("nt2", 0, 0), ("halo128", 2, 0), ("halo-nostag", 3, 0), ("halo", 1, 0), ("halo-4ph", 4, 0)]
if args.ablate:
    MODES += [("abl-noDMA", 1, 1), ("abl-noMFMA", 1, 2), ("abl-noLDSread", 1, 3)]


def timeit(fn, reps=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


for (name, H, W, C, K) in LAYERS:
    N = 4
    d = ops.conv_desc(N, H, W, C, K, 3, 3, dtype=ops.BF16)
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    wk = (torch.randn(K, 3, 3, C, device=dev) * 0.05).to(torch.bfloat16)
    wh = (torch.randn(3, 3, C, K, device=dev) * 0.05).to(torch.bfloat16)
    y = torch.empty(N, d.OH, d.OW, K, device=dev, dtype=torch.bfloat16)
    dx = torch.empty_like(x)
    flops = ops.conv_kernel_info(d, 0)[2]
    res = {}
    for rnd in range(4):
        for (m, halo, abl) in MODES:
            ops.set_option("nt_halo", 1 if halo else 0)
            ops.set_option("halo_wide", 0 if halo == 2 else 1)
            ops.set_option("halo_stagger", 0 if halo == 3 else 1)
            ops.set_option("halo_phases", 4 if halo == 4 else 2)
            ops.set_option("nt2_ablate", abl)
            res.setdefault((m, "fwd"), []).append(timeit(lambda: ops.conv2d_fwd(d, x, wk, y, None, ws)))
            if abl == 0:
                res.setdefault((m, "dgrad"), []).append(timeit(lambda: ops.conv2d_bwd_data(d, y, wh, dx, ws)))
    ops.set_option("nt_halo", 1)
    ops.set_option("nt2_ablate", 0)
    info = ops.conv_kernel_info(d, 0)[0], ops.conv_kernel_info(d, 1)[0]
    print(name, info, "  ".join(f"{m}/{k}={min(v)*1e3:.1f}us({flops/min(v)/1e9:.0f}TF)" for (m, k), v in res.items()),
          flush=True)

# ---- filter gradients: igemm_tn2 vs halo (NT 64 / 128)
WMODES = [("tn2", 0, 64), ("wgh64", 1, 64), ("wgh128", 1, 128)]
for (name, H, W, C, K) in LAYERS:
    N = 4
    d = ops.conv_desc(N, H, W, C, K, 3, 3, dtype=ops.BF16)
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    dy = torch.randn(N, H, W, K, device=dev).to(torch.bfloat16)
    dw = torch.empty(3, 3, C, K, device=dev, dtype=torch.float32)
    flops = ops.conv_kernel_info(d, 2)[2]
    res = {}
    for rnd in range(4):
        for (m, on, nt) in WMODES:
            ops.set_option("wgrad_halo", on)
            ops.set_option("wgrad_nt", nt)
            res.setdefault(m, []).append(timeit(lambda: ops.conv2d_bwd_filter(d, x, dy, dw, ws)))
    ops.set_option("wgrad_halo", 1)
    ops.set_option("wgrad_nt", 128)
    print(name, ops.conv_kernel_info(d, 2)[:2],
          "  ".join(f"{m}={min(v)*1e3:.1f}us({flops/min(v)/1e9:.0f}TF)" for m, v in res.items()), flush=True)
