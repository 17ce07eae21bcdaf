#!/bin/bash
# Round measurement: the driver's default bench line (C2 + C3 / C5 side lines, PMC traffic, CPU baseline),
# then rocprofv3 kernel traces of the same bench steps per config (timed-step stats: tools/timed_stats.py)
set -o pipefail
TAG=${1:-r05_m}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -30 $OUT/bench.err; exit 1; }
grep '^{' $OUT/bench.json | cut -c1-300
P="--no-cpu-baseline --no-traffic --no-miou --no-pipeline --no-extra --no-dp-probe --no-inference"
for m in fcn fcdensenet deeplab; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$m -o run -- python bench.py --model $m --steps 10 --warmup 3 $P > $OUT/prof_$m.json 2> $OUT/prof_$m.err || { echo rocprof $m failed; tail -20 $OUT/prof_$m.err; exit 1; }
done
echo done
