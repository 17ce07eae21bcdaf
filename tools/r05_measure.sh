#!/bin/bash
# Round measurement: the driver's default bench line (C2 + C3 / C5 side lines, PMC traffic, CPU baseline),
# then rocprofv3 kernel traces of the same bench steps per config (timed-step stats: tools/timed_stats.py)
set -o pipefail
TAG=${1:-r05_m}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -30 $OUT/bench.err; exit 1; }
grep '^{' $OUT/bench.json | cut -c1-300
P="--no-cpu-baseline --no-traffic --no-miou --no-pipeline --no-extra --no-dp-probe --no-inference"
# the C2 line (default steps) under a kernel trace: its roofline.avg_launch_ms against the trace of
# the same process's instrumented steps (tools/timed_stats.py --warmup W+K+2 --steps 5)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_line -o run -- python bench.py $P > $OUT/line_traced.json 2> $OUT/line_traced.err || { echo traced line failed; tail -20 $OUT/line_traced.err; exit 1; }
for m in fcn fcdensenet deeplab; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$m -o run -- python bench.py --model $m --steps 10 --warmup 3 $P > $OUT/prof_$m.json 2> $OUT/prof_$m.err || { echo rocprof $m failed; tail -20 $OUT/prof_$m.err; exit 1; }
done
echo done
