"""Time the FCN conv GEMMs (fwd / dgrad / wgrad) of one training step at the
bench shape, per kernel generation, interleaved in one process.
    python tools/convbench.py [--variants 1,2] [--reps 20]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semanticsegmentation_tensorflow_amd import ops  # noqa: E402

# (name, H, W, C, K, R) at batch 4, 384x1248
LAYERS = [("conv1_2", 384, 1248, 64, 64, 3), ("conv2_2", 192, 624, 128, 128, 3),
          ("conv3_2", 96, 312, 256, 256, 3), ("conv4_2", 48, 156, 512, 512, 3),
          ("conv5_2", 24, 78, 512, 512, 3), ("conv6", 12, 39, 512, 4096, 7), ("conv7", 12, 39, 4096, 4096, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="1,2")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=4)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    ws = ops.Workspace(dev)
    N = a.batch
    for (name, H, W, C, K, R) in LAYERS:
        d = ops.conv_desc(N, H, W, C, K, R, R, dtype=ops.BF16)
        x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
        wk = torch.randn(K, R, R, C, device=dev).to(torch.bfloat16) * 0.05
        wh = torch.randn(R, R, C, K, device=dev).to(torch.bfloat16) * 0.05
        y = torch.empty(N, d.OH, d.OW, K, device=dev, dtype=torch.bfloat16)
        dx = torch.empty_like(x)
        dw = torch.empty(R, R, C, K, device=dev)
        flops = ops.conv_kernel_info(d, 0)[2]
        for v in [int(s) for s in a.variants.split(",")]:
            ops.set_option("igemm_nt_variant", v)
            ops.set_option("igemm_tn_variant", v)
            res = []
            for op, fn in (("fwd", lambda: ops.conv2d_fwd(d, x, wk, y, ops.epilogue(relu=True), ws)),
                           ("dgrad", lambda: ops.conv2d_bwd_data(d, y, wh, dx, ws)),
                           ("wgrad", lambda: ops.conv2d_bwd_filter(d, x, y, dw, ws))):
                fn()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.reps):
                    fn()
                e.record()
                torch.cuda.synchronize()
                ms = s.elapsed_time(e) / a.reps
                kinfo = ops.conv_kernel_info(d, {"fwd": 0, "dgrad": 1, "wgrad": 2}[op])
                res.append(f"{op} {ms * 1e3:7.1f}us {flops / ms / 1e9:6.0f}TF {kinfo[0]}/s{kinfo[1]}")
            print(f"{name:8s} v{v}: " + " | ".join(res), flush=True)


if __name__ == "__main__":
    main()
