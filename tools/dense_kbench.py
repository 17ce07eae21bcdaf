"""Time the FC-DenseNet dense-layer launches (C3: bf16, batch 8) one at a
time with HIP events, interleaved over option sets in ONE process, and print
each one's algorithmic HBM bytes / time (Network/model/FCDenseNet.py:23-34:
BN -> ReLU -> 1x1 conv -> dropout -> BN -> ReLU -> 3x3 conv -> dropout).

    python tools/dense_kbench.py bn1x1:384:1248:128 bn3x3:384:1248 fwdbn2:384:1248:128 \
        grow:384:1248 smallk:384:1248:256

Specs (H, W at batch --batch; C = the concat-stack channels):
  bn1x1:H:W:C   input gradient of the bottleneck 1x1 conv (64 -> C) through
                the BN+ReLU before it, accumulated into the concat gradient
                (seg_conv2d_bwd_data_bn_part; bytes dy 64 + x C + old dx C + dx C)
  bn3x3:H:W     input gradient of the growth conv (16 -> 64) through BN+ReLU
                and the bottleneck's dropout (bytes dz 16 + x 64 + dx 64)
  fwdbn2:H:W:C  bottleneck forward: BN1 prologue, dropout, second output
                relu(BN2(y)) (bytes x C + y 64 + a 64)
  grow:H:W      growth conv forward 64 -> 16, dropout (bytes x 64 + y 16)
  smallk:H:W:C  final_conv input gradient 2 -> C with a ReluGrad mask
                (bytes dy 8 + mask C + dx C)
  wg3x3:H:W     growth conv filter gradient (bytes x 64 + dz 16)
  wg1x1:H:W:C   bottleneck filter gradient over relu(BN(x)) (bytes x C + dy 64)
A trailing ':nd' runs bn3x3 / fwdbn2 / grow without the dropout (its cost),
':nm' smallk without the mask; copy:H:W:C times torch's copy of C channels.
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semanticsegmentation_tensorflow_amd import ops  # noqa: E402

BF = torch.bfloat16


def setup(spec, N, dev, ws):
    kind, *dims = spec.split(":")
    nodrop = dims[-1] in ("nd", "nm")       # trailing ':nd' / ':nm': without dropout / mask
    dims = [int(v) for v in dims if v not in ("nd", "nm")]
    H, W = dims[0], dims[1]
    P = N * H * W
    g = torch.Generator(device=dev).manual_seed(1)

    def rnd(*shape, s=0.5):
        return (torch.randn(*shape, device=dev, generator=g) * s).to(BF)
    if kind == "bn1x1":
        C = dims[2]
        d = ops.conv_desc(N, H, W, C, 64, 1, 1, dtype=ops.BF16)
        dy, x, dx = rnd(N, H, W, 64), rnd(N, H, W, d.C), rnd(N, H, W, d.C)   # channels padded to 8
        w32 = torch.randn(1, 1, C, 64, device=dev, generator=g) / C ** 0.5
        wh = torch.zeros(ops.packed_shape(1, 1, C, 64, ops.PACK_HWIO, d.C), dtype=BF, device=dev)
        ops.pack_filter(w32, wh, d.C, 64, ops.PACK_HWIO)
        gm, bt = torch.ones(C, device=dev), torch.zeros(C, device=dev)

        def run():
            part = torch.empty(ops.conv_bwd_data_bn_part_rows(d) * 2 * d.C, device=dev)
            return lambda: ops.conv2d_bwd_data_bn_part(d, dy, wh, x, gm, bt, dx, part, accumulate=True)
        return d, ops.OP_BWD_DATA_BN, run, P * 2 * (64 + 3 * C)
    if kind == "bn3x3":
        d = ops.conv_desc(N, H, W, 64, 16, 3, 3, dtype=ops.BF16)
        dz, x, dx = rnd(N, H, W, 16), rnd(N, H, W, 64), torch.empty(N, H, W, 64, dtype=BF, device=dev)
        w32 = torch.randn(3, 3, 64, 16, device=dev, generator=g) / 24.0
        wh = torch.zeros(ops.packed_shape(3, 3, 64, 16, ops.PACK_HWIO, 64), dtype=BF, device=dev)
        ops.pack_filter(w32, wh, 64, 16, ops.PACK_HWIO)
        gm, bt = torch.ones(64, device=dev), torch.zeros(64, device=dev)

        def run():
            part = torch.empty(ops.conv_bwd_data_bn_part_rows(d) * 2 * 64, device=dev)
            return lambda: ops.conv2d_bwd_data_bn_part(d, dz, wh, x, gm, bt, dx, part,
                                                       dropout=None if nodrop else (0.2, 7))
        return d, ops.OP_BWD_DATA_BN, run, P * 2 * (16 + 64 + 64)
    if kind == "fwdbn2":
        C = dims[2]
        d = ops.conv_desc(N, H, W, C, 64, 1, 1, dtype=ops.BF16)
        x = rnd(N, H, W, d.C)
        w32 = torch.randn(1, 1, C, 64, device=dev, generator=g) / C ** 0.5
        wk = torch.zeros(ops.packed_shape(1, 1, C, 64, ops.PACK_KRSC, d.C), dtype=BF, device=dev)
        ops.pack_filter(w32, wk, d.C, 64, ops.PACK_KRSC)
        y, a = torch.empty(N, H, W, 64, dtype=BF, device=dev), torch.empty(N, H, W, 64, dtype=BF, device=dev)
        pro = ops.prologue(torch.ones(C, device=dev), torch.zeros(C, device=dev))
        g2, b2 = torch.ones(64, device=dev), torch.zeros(64, device=dev)
        epi = ops.epilogue(keep_prob=1.0 if nodrop else 0.2, seed=3)

        def run():
            return lambda: ops.conv2d_fwd_bn2(d, x, pro, wk, y, a, g2, b2, True, 1e-3, epi, ws)
        return d, ops.OP_FWD_PRO, run, P * 2 * (C + 128)
    if kind == "grow":
        d = ops.conv_desc(N, H, W, 64, 16, 3, 3, dtype=ops.BF16)
        x = rnd(N, H, W, 64)
        w32 = torch.randn(3, 3, 64, 16, device=dev, generator=g) / 24.0
        wk = torch.zeros(ops.packed_shape(3, 3, 64, 16, ops.PACK_KRSC, 64), dtype=BF, device=dev)
        ops.pack_filter(w32, wk, 64, 16, ops.PACK_KRSC)
        y = torch.empty(N, H, W, 16, dtype=BF, device=dev)
        epi = ops.epilogue(keep_prob=1.0 if nodrop else 0.2, seed=5)

        def run():
            return lambda: ops.conv2d_fwd(d, x, wk, y, epi, ws)
        return d, ops.OP_FWD, run, P * 2 * (64 + 16)
    if kind == "smallk":
        C = dims[2]
        d = ops.conv_desc(N, H, W, C, 2, 1, 1, dtype=ops.BF16)
        dy, mask = rnd(N, H, W, 8), torch.relu(rnd(N, H, W, C))
        w32 = torch.randn(1, 1, C, 2, device=dev, generator=g) / C ** 0.5
        wh = torch.zeros(ops.packed_shape(1, 1, C, 2, ops.PACK_HWIO, d.C), dtype=BF, device=dev)
        ops.pack_filter(w32, wh, d.C, d.K, ops.PACK_HWIO)
        dx = torch.empty(N, H, W, C, dtype=BF, device=dev)

        def run():
            return lambda: ops.conv2d_bwd_data(d, dy, wh, dx, ws, None,
                                               None if nodrop else ops.epilogue(relu_mask=mask))
        return d, ops.OP_BWD_DATA, run, P * 2 * (8 + (1 if nodrop else 2) * C)
    if kind == "wg3x3":                      # growth conv filter gradient (64 -> 16, 3x3)
        d = ops.conv_desc(N, H, W, 64, 16, 3, 3, dtype=ops.BF16)
        x, dz = rnd(N, H, W, 64), rnd(N, H, W, 16)
        dw = torch.empty(3, 3, 64, 16, device=dev)
        ws.get(ops.conv_workspace(d, ops.OP_BWD_FILTER))

        def run():
            return lambda: ops.conv2d_bwd_filter(d, x, dz, dw, ws)
        return d, ops.OP_BWD_FILTER, run, P * 2 * (64 + 16)
    if kind == "wg1x1":                      # bottleneck filter gradient over relu(BN(x)) (C -> 64)
        C = dims[2]
        d = ops.conv_desc(N, H, W, C, 64, 1, 1, dtype=ops.BF16)
        x, dy = rnd(N, H, W, d.C), rnd(N, H, W, 64)
        dw = torch.empty(1, 1, C, 64, device=dev)
        pro = ops.prologue(torch.ones(C, device=dev), torch.zeros(C, device=dev))
        ws.get(ops.conv_workspace(d, ops.OP_BWD_FILTER))

        def run():
            return lambda: ops.conv2d_bwd_filter_pro(d, x, pro, dy, dw, ws)
        return d, ops.OP_BWD_FILTER, run, P * 2 * (C + 64)
    if kind == "copy":                       # torch's elementwise copy: an HBM reference point
        C = dims[2]
        d = ops.conv_desc(N, H, W, C, 2, 1, 1, dtype=ops.BF16)
        src, dst = rnd(N, H, W, C), torch.empty(N, H, W, C, dtype=BF, device=dev)

        def run():
            return lambda: dst.copy_(src)
        return d, ops.OP_BWD_DATA, run, P * 2 * 2 * C
    raise SystemExit(f"unknown spec {spec}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("specs", nargs="+")
    ap.add_argument("--opts", action="append", default=None)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8)
    a = ap.parse_args()
    optsets = a.opts or [""]
    dev = torch.device("cuda:0")
    ws = ops.Workspace(dev)
    ws.get(1 << 26)
    cases = [setup(s, a.batch, dev, ws) for s in a.specs]

    def apply(o):
        for kv in filter(None, o.split(",")):
            k, v = kv.split("=")
            ops.set_option(k.strip(), int(v))

    times = {}
    for r in range(a.rounds):
        for oi, o in enumerate(optsets):
            apply(o)
            for ci, (d, op, make, nbytes) in enumerate(cases):
                fn = make()          # per option set: buffers sized for its launch geometry
                try:
                    fn()
                    torch.cuda.synchronize()
                except RuntimeError as err:
                    print(f"{a.specs[ci]} [{o}]: {err}", flush=True)
                    times.setdefault((ci, oi), []).append(float("nan"))
                    continue
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.reps):
                    fn()
                e.record()
                torch.cuda.synchronize()
                times.setdefault((ci, oi), []).append(s.elapsed_time(e) * 1e3 / a.reps)
        print(f"round {r + 1}/{a.rounds}", flush=True)
    for ci, (d, op, make, nbytes) in enumerate(cases):
        for oi, o in enumerate(optsets):
            apply(o)
            name = ops.conv_kernel_info(d, op)[0]
            t = times[(ci, oi)]
            if any(v != v for v in t):
                print(f"{a.specs[ci]:22s} [{o or 'default'}] {name:28s} failed")
                continue
            med = statistics.median(t)
            print(f"{a.specs[ci]:22s} [{o or 'default'}] {name:28s} med={med:8.1f}us min={min(t):8.1f}us  "
                  f"{nbytes / med / 1e3:7.1f} GB/s of {nbytes / 1e6:.0f} MB", flush=True)


if __name__ == "__main__":
    main()
