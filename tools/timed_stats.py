"""Kernel statistics of bench.py's TIMED steps only, from a rocprofv3
kernel-trace CSV of a bench run (`rocprofv3 --kernel-trace --stats
--output-format csv -- python bench.py --steps K --warmup W ...`).

    python tools/timed_stats.py TRACE_kernel_trace.csv --warmup W --steps K \
        [--family 'conv_halo2[<I]'] [--out profiles/X_timed_stats.csv]

Steps are delimited by the train step's input preparation kernel
(prepare_input_k, the first launch of every Session.run with a feed): the
W warm-up steps come first, then the K timed steps (bench.measure), so the
timed region is steps W .. W+K-1, each from its prepare_input to its last
adam_pack launch (--end-marker).
Prints (and with --out writes) rocprof-style per-kernel rows -- name, calls,
total / average / min / max ns -- for that region, and, with --family (a
bench.kernel_symbol pattern), the family's calls per step, average launch
duration and the roofline fraction it gives with bench.py's algorithmic
FLOPs per launch (--gflop) so the line's `frac` can be recomputed from the
committed summary."""
import argparse
import collections
import csv
import re
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--family", default=None)
    ap.add_argument("--gflop", type=float, default=None, help="algorithmic GFLOP per launch of the family")
    ap.add_argument("--gbytes", type=float, default=None, help="algorithmic GB per launch of the family (HBM bound)")
    ap.add_argument("--peak", type=float, default=2500.0, help="TFLOP/s (or GB/s with --gbytes)")
    ap.add_argument("--marker", default="prepare_input")
    ap.add_argument("--end-marker", default="adam_pack", help="last kernel of a train step")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(marks) < a.warmup + a.steps:
        sys.exit(f"{len(marks)} '{a.marker}' launches: fewer than warmup + steps")
    # each step: its input preparation .. its last Adam launch (the loss fetch
    # bench.py runs after the timed steps is not part of the last one)
    seg = []
    for j in range(a.warmup, a.warmup + a.steps):
        part = rows[marks[j]:marks[j + 1]] if j + 1 < len(marks) else rows[marks[j]:]
        last = max((i for i, r in enumerate(part) if a.end_marker in r["Kernel_Name"]), default=len(part) - 1)
        seg += part[:last + 1]
    t0 = int(seg[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in seg)
    agg = collections.OrderedDict()
    for r in seg:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        s = agg.setdefault(r["Kernel_Name"], [0, 0, None, 0])
        s[0] += 1
        s[1] += d
        s[2] = d if s[2] is None else min(s[2], d)
        s[3] = max(s[3], d)
    total = sum(v[1] for v in agg.values())
    out = [("Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs")]
    for k, (n, t, mn, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        out.append((k, n, t, round(t / n, 1), round(100.0 * t / total, 4), mn, mx))
    print(f"timed region: steps {a.warmup}..{a.warmup + a.steps - 1}, {len(seg)} dispatches, "
          f"wall {(t1 - t0) / 1e6:.3f} ms ({(t1 - t0) / 1e6 / a.steps:.3f} ms/step), kernel time {total / 1e6:.3f} ms")
    for row in out[:25]:
        print("  ".join(str(x) for x in row)[:160])
    if a.family:
        pat = re.compile(a.family)
        fam = [(k, v) for k, v in agg.items() if pat.search(k)]
        n = sum(v[0] for _, v in fam)
        t = sum(v[1] for _, v in fam)
        if n:
            avg_ms = t / n / 1e6
            line = f"family {a.family}: {n / a.steps:.1f} launches/step, avg {avg_ms * 1e3:.1f} us"
            if a.gflop:
                ach = a.gflop / avg_ms          # GFLOP per ms = TFLOP/s
                line += f", {ach:.1f} TFLOP/s = {ach / a.peak:.4f} of {a.peak:.0f}"
            if a.gbytes:
                ach = a.gbytes / avg_ms * 1e3    # GB/s
                line += f", {ach:.1f} GB/s = {ach / a.peak:.4f} of {a.peak:.0f}"
            print(line)
    if a.out:
        with open(a.out, "w", newline="") as f:
            csv.writer(f).writerows(out)


if __name__ == "__main__":
    main()
