"""Bit-compare one conv launch across kernel option sets (schedule variants
must not change a single output bit).
    python tools/variant_check.py conv4_2:fwd conv4_2:dgrad --opts 'x=0' --opts 'x=1'"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semanticsegmentation_tensorflow_amd import ops  # noqa: E402
from tools.kbench import LAYERS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("specs", nargs="+")
    ap.add_argument("--opts", action="append", default=[])
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    ws = ops.Workspace(dev)
    bad = 0
    for spec in a.specs:
        name, op = spec.split(":")
        H, W, C, K, R = LAYERS[name]
        N = 4
        d = ops.conv_desc(N, H, W, C, K, R, R, dtype=ops.BF16)
        g = torch.Generator(device=dev).manual_seed(5)
        x = (torch.randn(N, H, W, d.C, device=dev, generator=g)).to(torch.bfloat16)
        dy = (torch.randn(N, d.OH, d.OW, d.K, device=dev, generator=g)).to(torch.bfloat16)
        w32 = torch.randn(R, R, C, K, device=dev, generator=g) / (R * R * C) ** 0.5
        outs = []
        for o in a.opts:
            for kv in filter(None, o.split(",")):
                k, v = kv.split("=")
                ops.set_option(k, int(v))
            ws.get(ops.conv_workspace(d, ops.OP_FWD if op == "fwd" else ops.OP_BWD_DATA) + 1)
            if op == "fwd":
                wk = torch.zeros(ops.packed_shape(R, R, C, K, ops.PACK_KRSC, d.C), dtype=torch.bfloat16, device=dev)
                ops.pack_filter(w32, wk, d.C, d.K, ops.PACK_KRSC)
                y = torch.full((N, d.OH, d.OW, d.K), float("nan"), dtype=torch.bfloat16, device=dev)
                ops.conv2d_fwd(d, x, wk, y, ops.epilogue(bias=torch.zeros(K, device=dev), relu=True), ws)
            else:
                wh = torch.zeros(ops.packed_shape(R, R, C, K, ops.PACK_HWIO, d.C), dtype=torch.bfloat16, device=dev)
                ops.pack_filter(w32, wh, d.C, d.K, ops.PACK_HWIO)
                y = torch.full((N, H, W, d.C), float("nan"), dtype=torch.bfloat16, device=dev)
                ops.conv2d_bwd_data(d, dy, wh, y, ws)
            torch.cuda.synchronize()
            outs.append(y)
        for o, y in zip(a.opts[1:], outs[1:]):
            same = torch.equal(y.view(torch.int16), outs[0].view(torch.int16))
            bad += not same
            print(f"{spec:16s} [{o}] vs [{a.opts[0]}]: {'bit-identical' if same else 'DIFFERENT'} "
                  f"max|d|={(y.float() - outs[0].float()).abs().max().item():.3g}", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
