"""Time single conv launches of the C2 (FCN, bf16, batch 4, 384x1248) step
with HIP events, interleaved over option sets in ONE process (guide rule 24).

    python tools/kbench.py conv4_2:fwd conv3_2:dgrad conv6:wgrad ... \
        [--opts 'nt2_ablate=0'] [--opts 'nt2_ablate=1'] [--reps 20] [--rounds 5]

Option sets are applied in full before each use: give every set all the
knobs it changes (e.g. 'x=0' beside 'x=1').  Ablation knobs (*_abl,
nt2_ablate: garbage results) exist only in the diagnostic library: build it
with `_lib.build(diag=True)` and run with SEG_DIAG_LIB=1.

Each spec is LAYER:OP (OP fwd | dgrad | wgrad | wgrad_adam).  Prints, per
spec and option set, the median and min launch time (us) over rounds, the
kernel seg_conv_kernel_info names and TF/s at the median."""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semanticsegmentation_tensorflow_amd import ops  # noqa: E402

# (name, H, W, C, K, R) at 384x1248 (the C2 executed shape)
LAYERS = {"conv1_1": (384, 1248, 3, 64, 3), "conv1_2": (384, 1248, 64, 64, 3),
          "conv2_1": (192, 624, 64, 128, 3), "conv2_2": (192, 624, 128, 128, 3),
          "conv3_1": (96, 312, 128, 256, 3), "conv3_2": (96, 312, 256, 256, 3),
          "conv4_1": (48, 156, 256, 512, 3), "conv4_2": (48, 156, 512, 512, 3),
          "conv5_1": (24, 78, 512, 512, 3), "conv6": (12, 39, 512, 4096, 7), "conv7": (12, 39, 4096, 4096, 1)}
OPS = {"fwd": ops.OP_FWD, "dgrad": ops.OP_BWD_DATA, "dgradnm": ops.OP_BWD_DATA, "dgradbits": ops.OP_BWD_DATA,
       "wgrad": ops.OP_BWD_FILTER, "wgrad_adam": ops.OP_BWD_FILTER, "fwdbits": ops.OP_FWD, "fwdp": ops.OP_FWD, "dgradp": ops.OP_BWD_DATA, "fwdpool": ops.OP_FWD, "fwd+pool": ops.OP_FWD}
WPAD = 64   # fwdp / dgradp: packed filter rows padded by WPAD elements (diagnostic option "wpad")


def setup(spec, N, dev, ws):
    name, op = spec.split(":")
    H, W, C, K, R = LAYERS[name]
    d = ops.conv_desc(N, H, W, C, K, R, R, dtype=ops.BF16)
    g = torch.Generator(device=dev).manual_seed(1)
    x = (torch.randn(N, H, W, d.C, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    dy = (torch.randn(N, d.OH, d.OW, d.K, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    w32 = torch.randn(R, R, C, K, device=dev, generator=g) / (R * R * C) ** 0.5
    pad = WPAD if op.endswith("p") else 0

    def padded(fn):
        if not pad:
            return fn

        def run():
            ops.set_option("wpad", pad)
            fn()
            ops.set_option("wpad", 0)
        return run
    if op in ("fwd", "fwdp"):
        wk = torch.zeros(ops.packed_shape(R, R, C, K, ops.PACK_KRSC, d.C + pad), dtype=torch.bfloat16, device=dev)
        ops.pack_filter(w32, wk, d.C + pad, d.K, ops.PACK_KRSC)
        y = torch.empty(N, d.OH, d.OW, d.K, dtype=torch.bfloat16, device=dev)
        b = torch.zeros(K, device=dev)
        return d, op, padded(lambda: ops.conv2d_fwd(d, x, wk, y, ops.epilogue(bias=b, relu=True), ws))
    if op in ("fwdpool", "fwd+pool"):        # Conv2D + bias + ReLU + MaxPool 2x2: fused vs the pair
        wk = torch.zeros(ops.packed_shape(R, R, C, K, ops.PACK_KRSC, d.C), dtype=torch.bfloat16, device=dev)
        ops.pack_filter(w32, wk, d.C, d.K, ops.PACK_KRSC)
        y = torch.empty(N, d.OH, d.OW, d.K, dtype=torch.bfloat16, device=dev)
        yp = torch.empty(N, d.OH // 2, d.OW // 2, d.K, dtype=torch.bfloat16, device=dev)
        idx = torch.empty(N * (d.OH // 2) * (d.OW // 2) * d.K, dtype=torch.uint8, device=dev)
        b = torch.zeros(K, device=dev)
        epi = ops.epilogue(bias=b, relu=True)
        if op == "fwdpool":
            return d, op, lambda: ops.conv2d_fwd_pool(d, x, wk, yp, idx, epi, ws)

        def pair():
            ops.conv2d_fwd(d, x, wk, y, epi, ws)
            ops.maxpool2x2_fwd_argmax(y, yp, idx)
        return d, op, pair
    if op == "fwdbits":     # the forward that also writes its ReLU mask as bits
        wk = torch.zeros(ops.packed_shape(R, R, C, K, ops.PACK_KRSC, d.C), dtype=torch.bfloat16, device=dev)
        ops.pack_filter(w32, wk, d.C, d.K, ops.PACK_KRSC)
        y = torch.empty(N, d.OH, d.OW, d.K, dtype=torch.bfloat16, device=dev)
        bits = ops.relu_bits_buffer(N, d.OH, d.OW, d.K, dev)
        b = torch.zeros(K, device=dev)
        return d, op, lambda: ops.conv2d_fwd_relu_bits(d, x, wk, y, bits, ops.epilogue(bias=b, relu=True))
    if op == "dgradbits":   # the ReluGrad mask read as bits
        wh = torch.zeros(ops.packed_shape(R, R, C, K, ops.PACK_HWIO, d.C), dtype=torch.bfloat16, device=dev)
        ops.pack_filter(w32, wh, d.C, d.K, ops.PACK_HWIO)
        dx = torch.empty(N, H, W, d.C, dtype=torch.bfloat16, device=dev)
        bits = torch.randint(0, 256, (N, H, W, d.C // 8), dtype=torch.uint8, device=dev, generator=g)
        return d, op, lambda: ops.conv2d_bwd_data_bits(d, dy, wh, bits, dx, 1.0, ws)
    if op == "dgradnm":     # the input gradient without the ReluGrad mask epilogue
        wh = torch.zeros(ops.packed_shape(R, R, C, K, ops.PACK_HWIO, d.C), dtype=torch.bfloat16, device=dev)
        ops.pack_filter(w32, wh, d.C, d.K, ops.PACK_HWIO)
        dx = torch.empty(N, H, W, d.C, dtype=torch.bfloat16, device=dev)
        return d, op, lambda: ops.conv2d_bwd_data(d, dy, wh, dx, ws, None, None)
    if op in ("dgrad", "dgradp"):
        wh = torch.zeros(ops.packed_shape(R, R, C, K + pad, ops.PACK_HWIO, d.C), dtype=torch.bfloat16, device=dev)
        ops.pack_filter(w32, wh, d.C, d.K + pad, ops.PACK_HWIO)
        dx = torch.empty(N, H, W, d.C, dtype=torch.bfloat16, device=dev)
        mask = torch.relu(torch.randn(N, H, W, d.C, device=dev, generator=g)).to(torch.bfloat16)
        return d, op, padded(lambda: ops.conv2d_bwd_data(d, dy, wh, dx, ws, None, ops.epilogue(relu_mask=mask)))
    dw = torch.empty(R, R, C, K, device=dev)
    db = torch.empty(K, device=dev)
    if op == "wgrad":
        return d, op, lambda: ops.conv2d_bwd_filter(d, x, dy, dw, ws, None, db)
    p = w32.clone()
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    wh = torch.zeros(ops.packed_shape(R, R, C, K, ops.PACK_HWIO, d.C), dtype=torch.bfloat16, device=dev)
    wk = torch.zeros(ops.packed_shape(R, R, C, K, ops.PACK_KRSC, d.C), dtype=torch.bfloat16, device=dev)
    hw = (wh, d.C, d.K)
    kr = (wk, d.C, d.K)
    return d, op, lambda: ops.conv2d_bwd_filter_adam(d, x, dy, p, m, v, 1e-4, 1, 0.9, 0.999, 1e-8, 1.0, hw, kr,
                                                     None, db, ws)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("specs", nargs="+")
    ap.add_argument("--opts", action="append", default=None)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--batch", type=int, default=4)
    a = ap.parse_args()
    optsets = a.opts or [""]
    dev = torch.device("cuda:0")
    ws = ops.Workspace(dev)
    cases = [setup(s, a.batch, dev, ws) for s in a.specs]
    need = max(ops.conv_workspace(d, OPS[op]) for d, op, _ in cases)
    ws.get(max(need, 1 << 20))

    def apply(o):
        for kv in filter(None, o.split(",")):
            k, v = kv.split("=")
            ops.set_option(k.strip(), int(v))

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
            print(f"{a.specs[ci]:16s} [{o or 'default'}] {name:28s} splits={splits:<3d} "
                  f"med={med:8.1f}us min={min(t):8.1f}us  {flops / med / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
