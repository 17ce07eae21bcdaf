"""Time single launches of C3's decoder transposed convolutions (FC-DenseNet
transition_up1..5 at batch 8, 384x1248: Network/model/FCDenseNet.py:141-154)
with HIP events, interleaved over option sets in ONE process (as kbench.py).

    python tools/tconv_kbench.py up5:fwd up5:dgrad up3:dgrad ... \
        [--opts 'nt_nsplit=1'] [--opts 'nt_nsplit=0'] [--reps 10] [--rounds 5]

OP: fwd (Conv2DTranspose), dgrad (its input gradient), wgrad (its filter
gradient).  Prints, per spec and option set, the median / min launch time,
the kernel seg_conv_kernel_info names and TF/s at the median.  As in
kbench.py, give every option set all the knobs any set changes (knobs are
process-global: a set that omits one runs with the value the previous set
left).  Round-5 results: profiles/r05_c3_decoder_kbench.txt."""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semanticsegmentation_tensorflow_amd import ops  # noqa: E402

# (IH, IW, Ci, OH, OW, Co): input / output of the 4x4 stride-2 transposed conv
UPS = {"up1": (12, 39, 430, 24, 78, 348), "up2": (24, 78, 696, 48, 156, 280),
       "up3": (48, 156, 560, 96, 312, 208), "up4": (96, 312, 416, 192, 624, 160),
       "up5": (192, 624, 320, 384, 1248, 128)}
OPS = {"fwd": ops.OP_TFWD, "dgrad": ops.OP_TBWD_DATA, "wgrad": ops.OP_TBWD_FILTER}


def setup(spec, N, dev, ws):
    name, op = spec.split(":")
    IH, IW, Ci, OH, OW, Co = UPS[name]
    d = ops.tconv_desc(N, IH, IW, Ci, OH, OW, Co, 4, 4, 2, "SAME", ops.BF16)
    g = torch.Generator(device=dev).manual_seed(1)
    x = (torch.randn(N, IH, IW, d.C, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    dy = (torch.randn(N, OH, OW, d.K, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    w32 = torch.randn(4, 4, Co, Ci, device=dev, generator=g) / (4 * Ci) ** 0.5
    ap = ops.tconv_filter_apad(d)
    if op == "fwd":
        wp = torch.empty(ops.packed_shape(4, 4, Co, Ci, ops.PACK_TCONV_FWD, ap), dtype=torch.bfloat16, device=dev)
        ops.pack_filter(w32, wp, ap, ops.round8(Ci), ops.PACK_TCONV_FWD)
        y = torch.empty(N, OH, OW, d.K, dtype=torch.bfloat16, device=dev)
        b = torch.zeros(Co, device=dev)
        return d, op, lambda: ops.tconv2d_fwd(d, x, wp, y, ops.epilogue(bias=b), ws)
    if op == "dgrad":
        wb = torch.empty(ops.packed_shape(4, 4, Co, Ci, ops.PACK_TCONV_BWD, ap), dtype=torch.bfloat16, device=dev)
        ops.pack_filter(w32, wb, ap, ops.round8(Ci), ops.PACK_TCONV_BWD)
        dx = torch.empty(N, IH, IW, d.C, dtype=torch.bfloat16, device=dev)
        return d, op, lambda: ops.tconv2d_bwd_data(d, dy, wb, dx, ws)
    dw = torch.empty(4, 4, Co, Ci, device=dev)
    db = torch.empty(Co, device=dev)
    return d, op, lambda: ops.tconv2d_bwd_filter(d, x, dy, dw, ws, None, db)


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

    def apply(o):
        for kv in filter(None, o.split(",")):
            k, v = kv.split("=")
            ops.set_option(k.strip(), int(v))

    cases = [setup(s, a.batch, dev, ws) for s in a.specs]
    need = 0
    for o in optsets:
        apply(o)
        need = max([need] + [ops.conv_workspace(d, OPS[op]) for d, op, _ in cases])
    ws.get(max(need, 1 << 20))
    times = {}
    for r in range(a.rounds):
        for oi, o in enumerate(optsets):
            apply(o)
            for ci, (d, op, fn) in enumerate(cases):
                fn()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.reps):
                    fn()
                e.record()
                torch.cuda.synchronize()
                times.setdefault((ci, oi), []).append(s.elapsed_time(e) * 1e3 / a.reps)
    for ci, (d, op, fn) in enumerate(cases):
        for oi, o in enumerate(optsets):
            apply(o)
            name, splits, flops = ops.conv_kernel_info(d, OPS[op])
            t = times[(ci, oi)]
            med = statistics.median(t)
            print(f"{a.specs[ci]:10s} [{o or 'default'}] {name:28s} splits={splits:<3d} "
                  f"med={med:8.1f}us min={min(t):8.1f}us  {flops / med / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
