#!/bin/bash
# A/B of the C2 step: bench.py (headline only) under several argument sets.
# usage: tools/ab_bench.sh TAG "ARGS1" "ARGS2" ...
#   (each e.g. "--schedule side_wgrad=1 --option tn_fill=2", or "" for the defaults)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
Q="--steps 30 --warmup 5 --no-cpu-baseline --no-traffic --no-miou --no-pipeline --no-extra --no-dp-probe --no-inference"
i=0
for rep in 1 2; do
  for e in "$@"; do
    i=$((i+1))
    timeout -k 10 200 python bench.py $Q $BENCH_ARGS $e > $OUT/b$i.json 2> $OUT/b$i.err || { echo "bench failed: $e"; tail -20 $OUT/b$i.err; exit 1; }
    python -c "import json,sys; d=[json.loads(l) for l in open('$OUT/b$i.json') if l.startswith('{')][-1]; print('%-45s %8.1f img/s %6.3f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$e"
  done
done
