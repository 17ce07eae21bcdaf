"""Per-kernel time of ONE timed step from a rocprofv3 kernel-trace CSV of a
bench run, side by side for two traces (e.g. the serialised step,
--schedule side_wgrad=0, against the default overlapped one):

    python tools/step_families.py SERIAL.csv OVERLAP.csv --warmup 3 --steps 5

Steps run from the input-preparation kernel to the step's last Adam launch;
the per-step average over the timed steps is printed per kernel symbol
(shortened), with the step wall time of each trace."""
import argparse
import collections
import csv
import re


def step_rows(rows, marks, j, end_marker="adam_pack"):
    """Dispatches of train step j: from its input preparation up to its last
    Adam launch (what follows before the next step -- bench.py's loss fetch
    after the timed steps -- is not part of it)."""
    seg = rows[marks[j]:marks[j + 1]] if j + 1 < len(marks) else rows[marks[j]:]
    last = max((i for i, r in enumerate(seg) if end_marker in r["Kernel_Name"]), default=len(seg) - 1)
    return seg[:last + 1]


def per_step(path, warmup, steps, marker="prepare_input"):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    seg = [r for j in range(warmup, warmup + steps) for r in step_rows(rows, marks, j)]
    wall = sum(max(int(r["End_Timestamp"]) for r in step_rows(rows, marks, j)) -
               int(rows[marks[j]]["Start_Timestamp"]) for j in range(warmup, warmup + steps)) / 1e3 / steps
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in seg:
        k = short(r["Kernel_Name"])
        agg[k][0] += 1
        agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return wall, {k: (n / steps, t / steps) for k, (n, t) in agg.items()}


def short(name):
    name = re.sub(r"^_ZN\d+seg\d+|^_ZN\d+_GLOBAL__N_1\d+|^_Z\d+", "", name)
    return name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--top", type=int, default=30)
    x = ap.parse_args()
    wa, a = per_step(x.a, x.warmup, x.steps)
    wb, b = per_step(x.b, x.warmup, x.steps)
    print(f"step wall: {wa / 1e3:.3f} ms | {wb / 1e3:.3f} ms; kernel time {sum(v[1] for v in a.values()) / 1e3:.3f} | "
          f"{sum(v[1] for v in b.values()) / 1e3:.3f} ms")
    keys = sorted(set(a) | set(b), key=lambda k: -a.get(k, (0, 0))[1])
    for k in keys[:x.top]:
        na, ta = a.get(k, (0, 0.0))
        nb, tb = b.get(k, (0, 0.0))
        print(f"{ta:9.1f} {tb:9.1f} us  n={na:5.1f}  {k}")


if __name__ == "__main__":
    main()
