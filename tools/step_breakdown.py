"""Per-step kernel breakdown from a rocprofv3 kernel-trace CSV: one steady-state
step = the launches between the last two Adam launches."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"]]
b = idx[-1]
# the train step starts at its input preparation (the last one before Adam)
a = max(i for i in range(b) if "prepare_input" in rows[i]["Kernel_Name"]) - 1
step = rows[a + 1:b + 1]
t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
print(f"step wall {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, {len(step)} kernels")
agg, cnt = collections.defaultdict(float), collections.Counter()
for r in step:
    n = r["Kernel_Name"]
    n = re.sub(r"^void ", "", n)
    k = re.sub(r"\(.*", "", n)[:70] or n[:70]
    agg[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    cnt[k] += 1
for k, v in sorted(agg.items(), key=lambda x: -x[1]):
    print(f"{v:9.1f} {cnt[k]:4d} {k}")
if len(sys.argv) > 2:
    print("--- launches in order ---")
    for r in step:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        print(f"{d:8.1f} {r['Kernel_Name'][:90]}")
