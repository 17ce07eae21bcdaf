"""Can a register-light, LDS-free TF1 Adam stream (seg_adam_tf1_shadow) run
BESIDE the MFMA-bound conv kernels?  Times, in one process:
  (1) N launches of a C2 conv kernel alone (kbench's setup),
  (2) the shadow Adam over conv6's 102.8 M parameters alone,
  (3) both together on two streams: the conv launches' time and the Adam's.
usage: python tools/shadow_probe.py conv4_2:fwd conv3_2:dgrad conv4_2:wgrad [--reps 20] [--blocks 256]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semanticsegmentation_tensorflow_amd import ops  # noqa: E402
from tools.kbench import setup, OPS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("specs", nargs="+")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--blocks", type=int, default=256)
    ap.add_argument("--n", type=int, default=102760448)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    ws = ops.Workspace(dev)
    n = a.n
    p = torch.randn(n, device=dev) * 0.01
    g = torch.randn(n, device=dev) * 1e-3
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    c16 = torch.empty(n, dtype=torch.bfloat16, device=dev)
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def adam(blocks):
        ops.adam_tf1_shadow(p, g, m, v, 1e-4, 1, copy16=c16, blocks=blocks, stream=sb)

    def ev():
        return torch.cuda.Event(enable_timing=True)
    for blocks in (a.blocks, 2 * a.blocks, 4096):
        with torch.cuda.stream(sb):
            adam(blocks)
            torch.cuda.synchronize()
            s, e = ev(), ev()
            s.record(sb)
            adam(blocks)
            e.record(sb)
        torch.cuda.synchronize()
        dt = s.elapsed_time(e) * 1e3
        print(f"shadow adam alone, {blocks} blocks: {dt:8.1f} us  {n * 30 / dt / 1e6:7.1f} GB/s (30 B/param)",
              flush=True)
    for spec in a.specs:
        d, op, fn = setup(spec, 4, dev, ws)
        ws.get(max(ops.conv_workspace(d, OPS[op]), 1 << 20))
        name = ops.conv_kernel_info(d, OPS[op])[0]
        with torch.cuda.stream(sa):
            fn()
            torch.cuda.synchronize()
            s, e = ev(), ev()
            s.record(sa)
            for _ in range(a.reps):
                fn()
            e.record(sa)
            torch.cuda.synchronize()
            alone = s.elapsed_time(e) * 1e3 / a.reps
            # together: the Adam first on stream b, then the conv launches on a
            s2, e2, sb0, eb0 = ev(), ev(), ev(), ev()
            sb0.record(sb)
            with torch.cuda.stream(sb):
                adam(a.blocks)
            eb0.record(sb)
            s2.record(sa)
            for _ in range(a.reps):
                fn()
            e2.record(sa)
            torch.cuda.synchronize()
            both = s2.elapsed_time(e2) * 1e3 / a.reps
            adam_t = sb0.elapsed_time(eb0) * 1e3
        print(f"{spec:16s} {name:26s} alone {alone:8.1f} us/launch | beside the Adam {both:8.1f} us/launch "
              f"(x{both / alone:.3f}); Adam took {adam_t:8.1f} us over {a.reps} launches = "
              f"{a.reps * both:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
