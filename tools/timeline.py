"""Per-step timeline from a rocprofv3 kernel-trace CSV: one steady-state step
(between two input preparations), main vs side queue, grouped by kernel."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
which = int(sys.argv[2]) if len(sys.argv) > 2 else -5   # a timed step (later windows hold plan compiles)
pi = [i for i, r in enumerate(rows) if "prepare_input" in r["Kernel_Name"]]
a, b = pi[which - 1], pi[which]
step = rows[a:b]
t0 = int(step[0]["Start_Timestamp"])
print("wall us", (int(rows[b]["Start_Timestamp"]) - t0) / 1e3)
agg = collections.defaultdict(lambda: [0, 0.0])
for r in step:
    n = re.sub(r"^void ", "", r["Kernel_Name"])
    n = re.sub(r"\(.*", "", n)[:70] or r["Kernel_Name"][:70]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    a_ = agg[(r["Queue_Id"], n)]
    a_[0] += 1
    a_[1] += d
for (q, n), (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"q{q} {d:9.1f} {c:4d} {n}")
