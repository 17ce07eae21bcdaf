#!/bin/bash
# round-5 probe: C2 bench at the box's GPU_MAX_HW_QUEUES (4) and at 8, plus a
# kernel trace of the bench's own steps.   usage: tools/r05_probe.sh TAG
set -o pipefail
TAG=${1:-r05_a}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
B="--no-extra --no-traffic --no-cpu-baseline --no-pipeline --no-inference --no-miou --kernel-table"
echo "HWQ=$GPU_MAX_HW_QUEUES"
timeout -k 10 300 python bench.py $B "$@" > $OUT/hwq4.json 2> $OUT/hwq4.err || { echo bench4 failed; tail -20 $OUT/hwq4.err; exit 1; }
cut -c1-400 $OUT/hwq4.json
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py $B "$@" > $OUT/hwq8.json 2> $OUT/hwq8.err || { echo bench8 failed; tail -20 $OUT/hwq8.err; exit 1; }
cut -c1-400 $OUT/hwq8.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 10 --warmup 3 $B --no-dp-probe "$@" > $OUT/prof.json 2> $OUT/prof.err || { echo rocprof failed; tail -20 $OUT/prof.err; exit 1; }
echo done
