"""Per-launch conv census of a bench training step, on the CPU (no GPU).

Builds the bench.py training graph (same Session, same schedule) over a
recording stub of the C-ABI, runs one train step without computing anything,
and lists every conv / conv2d_transpose launch with the kernel family the
library's planner picks for it (seg_conv_kernel_info, host-only), its split-K
factor and its algorithmic GFLOP -- the map from a rocprof kernel trace back
to the model's layers.

    python tools/conv_census.py [--model fcdensenet] [--batch 8] [--top 40]
"""
import argparse
import collections
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from semanticsegmentation_tensorflow_amd import _lib, ops  # noqa: E402

OPCODE = {"seg_conv2d_fwd": 0, "seg_conv2d_fwd_pool": 0, "seg_conv2d_fwd_bn2": 0, "seg_conv2d_fwd_bn2_pro": 7, "seg_conv2d_bwd_data": 1, "seg_conv2d_bwd_filter": 2,
          "seg_conv2d_bwd_filter_begin": 2, "seg_conv2d_bwd_filter_adam": 2, "seg_tconv2d_fwd": 3,
          "seg_tconv2d_bwd_data": 4, "seg_tconv2d_bwd_filter": 5, "seg_conv2d_bwd_data_bn": 6,
          "seg_conv2d_fwd_pro": 7, "seg_conv2d_bwd_filter_pro": 8}
OPNAME = ["fwd", "dgrad", "wgrad", "tfwd", "tdgrad", "twgrad", "dgrad_bn", "fwd_pro", "wgrad_pro"]
HOST_ONLY = ("seg_conv_desc_init", "seg_tconv_desc_init", "seg_conv_workspace", "seg_bias_grad_workspace",
             "seg_xent_workspace", "seg_status_string", "seg_adam_segments_plan", "seg_tconv_filter_apad",
             "seg_conv_wgrad_adam_fusable", "seg_conv_bwd_data_bn_workspace", "seg_conv2d_fwd_pool_ok",
             "seg_conv_kernel_info", "seg_conv2d_fwd_bn2_ok")


class Recorder:
    def __init__(self, real):
        self.real = real
        self.launches = []
        self.calls = []

    def __getattr__(self, name):
        real_fn = getattr(self.real, name)

        def fn(*a):
            if name in HOST_ONLY:
                return real_fn(*a)
            self.calls.append(name)
            if name in OPCODE:
                d = _lib.SegConvDesc()
                ctypes.pointer(d)[0] = a[0]._obj
                pro = name == "seg_conv2d_fwd_bn2" and a[2] is not None   # BN1 prologue: the FWD_PRO plan
                self.launches.append((name + ("_pro" if pro else ""), d))
            return 0
        return fn


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="fcdensenet")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--pflops", type=float, default=1.25, help="rate for the 'ideal us' column")
    ap.add_argument("--fills", action="store_true",
                    help="also list the torch zero-fills / allocations a steady-state step issues, by call site")
    a = ap.parse_args()
    import bench
    H, W, B, kp = bench.DEFAULTS[a.model]
    B = a.batch or B
    rec = Recorder(_lib.load())
    _lib.lib = lambda: rec
    ops.stream_ptr = lambda s=None: None
    torch.cuda.is_available = lambda: True
    from semanticsegmentation_tensorflow_amd import session as S
    orig_init = S.Session.__init__

    def init(self, *args, **kw):
        kw["device"] = torch.device("cpu")
        orig_init(self, *args, **kw)
    S.Session.__init__ = init
    g = bench.build_train_graph(a.model, H, W, bench.DEFAULT_DTYPE[a.model])
    HP, WP = g["HP"], g["WP"]
    feed = {g["image"]: np.zeros((B, HP, WP, 3), np.float32), g["labels"]: np.zeros((B, HP, WP), np.uint8),
            g["keep"]: kp}
    g["sess"].run(g["train_step"], feed_dict=feed)    # first step: one-time filter packing
    rec.launches.clear()
    rec.calls.clear()
    fills = collections.Counter()
    if a.fills:
        import traceback

        def site():
            for fr in reversed(traceback.extract_stack()[:-2]):
                if "semanticsegmentation_tensorflow_amd" in fr.filename:
                    return f"{os.path.basename(fr.filename)}:{fr.lineno}"
            return "?"

        def wrap(obj, name):
            orig = getattr(obj, name)

            def fn(*args, **kw):
                out = orig(*args, **kw)
                t = out if isinstance(out, torch.Tensor) else None
                fills[(name, site())] += t.numel() * t.element_size() if t is not None else 0
                return out
            setattr(obj, name, fn)
        for n in ("zero_", "fill_"):
            wrap(torch.Tensor, n)
        for n in ("zeros", "zeros_like", "empty", "empty_like", "full", "full_like"):
            wrap(torch, n)
    g["sess"].run(g["train_step"], feed_dict=feed)
    if a.fills:
        print("torch allocations / fills in a steady-state step (bytes by call site):")
        for (n, s), b in fills.most_common():
            print(f"  {n:12s} {s:28s} {b / 1e6:10.1f} MB")
    rows = collections.OrderedDict()
    total = 0.0
    for name, d in rec.launches:
        op = OPCODE[name]
        kern, splits, flops = ops.conv_kernel_info(d, op)
        key = (OPNAME[op] + ("+pool" if name.endswith("_pool") else ""), kern, splits,
               f"{d.N}x{d.H}x{d.W}x{d.c_valid}->{d.OH}x{d.OW}x{d.k_valid} {d.R}x{d.S}/{d.stride_h}")
        r = rows.setdefault(key, [0, 0.0])
        r[0] += 1
        r[1] += flops
        total += flops
    print(f"{a.model} batch {B} at {HP}x{WP}: {len(rec.launches)} conv launches, {total / 1e9:.1f} GFLOP "
          f"({total / 1e9 / (a.pflops * 1e3):.2f} ms at {a.pflops} PF/s)")
    fam = collections.defaultdict(lambda: [0, 0.0])
    for (op, kern, splits, shape), (n, fl) in rows.items():
        fam[(op, kern)][0] += n
        fam[(op, kern)][1] += fl
    print("\nby op / kernel family:")
    for (op, kern), (n, fl) in sorted(fam.items(), key=lambda x: -x[1][1]):
        print(f"  {op:10s} {kern:28s} {n:4d} launches {fl / 1e9:9.1f} GFLOP")
    print("\nC-ABI calls per step:", dict(collections.Counter(rec.calls).most_common()))
    print(f"\ntop {a.top} launch shapes by GFLOP:")
    for (op, kern, splits, shape), (n, fl) in sorted(rows.items(), key=lambda x: -x[1][1])[:a.top]:
        print(f"  {n:3d}x {op:10s} {kern:24s} s={splits:<3d} {shape:44s} {fl / 1e9 / n:8.2f} GF "
              f"ideal {fl / n / (a.pflops * 1e15) * 1e6:7.1f} us")


if __name__ == "__main__":
    main()
