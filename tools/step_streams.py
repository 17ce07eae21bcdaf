"""Per-stream kernel breakdown of one steady-state step from a rocprofv3
kernel-trace CSV (how profiles/r04_*_step_kernels.txt were made).

    python tools/step_streams.py TRACE.csv MARKER [K]

MARKER: a substring of a kernel launched once per step (e.g. 'smallk' for
C3, 'adam_pack' for C2); the step is the launches after the K-1-th marker up
to and including the K-th (default K = 3).  Prints the step's wall time, the
busy time per HIP stream and the kernel families by total time with their
launch counts per stream."""
import csv, sys, collections, re
path=sys.argv[1]; marker=sys.argv[2]; k=int(sys.argv[3]) if len(sys.argv)>3 else 3
rows=list(csv.DictReader(open(path)))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
marks=[i for i,r in enumerate(rows) if marker in r['Kernel_Name']]
seg=rows[marks[k-1]+1:marks[k]+1]
t0=int(seg[0]['Start_Timestamp']); t1=max(int(r['End_Timestamp']) for r in seg)
print(f"step wall {(t1-t0)/1e3:.0f} us, {len(seg)} kernels")
bys=collections.defaultdict(float)
for r in seg: bys[r['Stream_Id']]+= (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3
print("per stream busy us:", {s:round(v) for s,v in bys.items()})
agg=collections.defaultdict(lambda:[0,0.0,collections.Counter()])
def short(n):
    n=re.sub(r'\(.*','',n); return n[:70]
for r in seg:
    d=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3
    a=agg[short(r['Kernel_Name'])]; a[0]+=1; a[1]+=d; a[2][r['Stream_Id']]+=1
for n,(c,d,s) in sorted(agg.items(), key=lambda x:-x[1][1])[:40]:
    print(f"{d:8.0f} us {c:4d} {d/c:8.1f} {dict(s)} {n}")
