"""Per-kernel HBM traffic of the last train step from bench.py's PMC child
passes (gpurun_out/bench_pmc/{fetch_size,write_size}) -> CSV on stdout.
FETCH_SIZE / WRITE_SIZE are KiB as rocprofv3 reports them (apply the gfx950
x2 FETCH_SIZE correction when comparing with byte counts)."""
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/bench_pmc"
print("counter,kernel,dispatches,total_kib_last_step")
for c in ("fetch_size", "write_size"):
    f = glob.glob(f"{root}/{c}/**/*counter_collection.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
    st = [i for i, r in enumerate(rows) if "prepare_input" in r["Kernel_Name"]][-1]
    agg = {}
    for r in rows[st:]:
        k = r["Kernel_Name"][:80].replace(",", ";")
        a = agg.setdefault(k, [0, 0.0])
        a[0] += 1
        a[1] += float(r["Counter_Value"])
    for k, (n, v) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{c.upper()},{k},{n},{v:.0f}")
