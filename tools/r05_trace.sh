#!/bin/bash
# rocprofv3 kernel traces of bench steps: r05_trace.sh TAG "name|model|extra bench args" ...
set -o pipefail
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
P="--no-cpu-baseline --no-traffic --no-miou --no-pipeline --no-extra --no-dp-probe --no-inference --steps 5 --warmup 3"
for spec in "$@"; do
  IFS='|' read -r name model args <<< "$spec"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$name -o run -- python bench.py --model $model $P $args > $OUT/prof_$name.json 2> $OUT/prof_$name.err || { echo rocprof $name failed; tail -20 $OUT/prof_$name.err; exit 1; }
  echo "$name traced"
done
echo done
