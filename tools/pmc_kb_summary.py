"""Per-kernel mean counter values over the dispatches of tools/pmc_kb.sh's
passes (OUTDIR/p1..p3), plus derived ratios: MFMA busy share of the
wave-cycle budget, waits per wave-cycle, VALU per MFMA, L2 hit rate,
effective clock (GRBM_GUI_ACTIVE / 8 / duration)."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:60]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in glob.glob(f"{root}/p*/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Kernel_Name"][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, c in vals.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    d = sum(dur[k]) / max(1, len(dur[k]))
    if d < 5:
        continue
    print(f"== {k}  dispatches~{len(next(iter(c.values())))}  avg {d:.1f} us")
    for n in sorted(m):
        print(f"   {n:28s} {m[n]:.4g}")
    g = lambda n: m.get(n, 0.0)   # noqa: E731
    if g("SQ_INSTS_MFMA"):
        print(f"   VALU/MFMA {g('SQ_INSTS_VALU') / g('SQ_INSTS_MFMA'):.2f}  LDS/MFMA {g('SQ_INSTS_LDS') / g('SQ_INSTS_MFMA'):.2f}")
    if g("SQ_WAVE_CYCLES"):
        print(f"   wait_any/wave_cycles {g('SQ_WAIT_ANY') / g('SQ_WAVE_CYCLES'):.3f}  "
              f"wait_inst/wave_cycles {g('SQ_WAIT_INST_ANY') / g('SQ_WAVE_CYCLES'):.3f}")
    if g("TCC_HIT_sum") + g("TCC_MISS_sum"):
        print(f"   L2 hit {g('TCC_HIT_sum') / (g('TCC_HIT_sum') + g('TCC_MISS_sum')):.3f}")
    if g("GRBM_GUI_ACTIVE"):
        print(f"   clock ~{g('GRBM_GUI_ACTIVE') / 8 / (d * 1e-6) / 1e9:.2f} GHz")
    if g("SQ_VALU_MFMA_BUSY_CYCLES") and g("GRBM_GUI_ACTIVE"):
        print(f"   MFMA busy share {g('SQ_VALU_MFMA_BUSY_CYCLES') / (g('GRBM_GUI_ACTIVE') / 8 * 256 * 4):.3f}")
