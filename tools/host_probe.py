"""Host-side cost of a bench training step: how long sess.run(train_step)
takes to ENQUEUE (no synchronisation) against the GPU time of the step.  If
the enqueue time approaches the step time, the step is launch-bound.

    python tools/host_probe.py [--model fcn] [--steps 6]

Prints per-step enqueue ms (the GPU is kept busy by the previous steps, so
the queue never drains), the synchronised ms/step, and a cProfile summary of
one step's host time (top functions by cumulative time)."""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="fcn")
    ap.add_argument("--steps", type=int, default=6)
    a = ap.parse_args()
    H, W, B, kp = bench.DEFAULTS[a.model]
    dev = torch.device("cuda:0")
    g = bench.build_train_graph(a.model, H, W, bench.DEFAULT_DTYPE[a.model])
    sess = g["sess"]
    img, lab = bench.synthetic(B, H, W, g["HP"], g["WP"], 1234, dev)
    feed = {g["image"]: img, g["labels"]: lab, g["keep"]: kp}
    for _ in range(3):
        sess.run(g["train_step"], feed_dict=feed)
    torch.cuda.synchronize()
    enq = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        t = time.perf_counter()
        sess.run(g["train_step"], feed_dict=feed)
        enq.append((time.perf_counter() - t) * 1e3)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{a.model}: enqueue ms/step {[round(e, 2) for e in enq]}; loop {1e3 * (t1 - t0) / a.steps:.2f} ms/step, "
          f"with the final sync {1e3 * (t2 - t0) / a.steps:.2f} ms/step", flush=True)
    pr = cProfile.Profile()
    torch.cuda.synchronize()
    pr.enable()
    sess.run(g["train_step"], feed_dict=feed)
    pr.disable()
    torch.cuda.synchronize()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(25)
    print(s.getvalue())


if __name__ == "__main__":
    main()
