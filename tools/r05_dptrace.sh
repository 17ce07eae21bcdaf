#!/bin/bash
# C2 line with the world-1 RCCL data-parallel probe, under a kernel trace
set -o pipefail
TAG=${1:-r05_s}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
B="--no-extra --no-traffic --no-cpu-baseline --no-pipeline --no-inference --no-miou --steps 10 --warmup 3"
timeout -k 10 400 python bench.py $B > $OUT/dp_plain.json 2> $OUT/dp_plain.err || { echo plain failed; tail -20 $OUT/dp_plain.err; exit 1; }
grep -h '^{' $OUT/dp_plain.json | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print('plain', d['value'], d['dp_mode'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_dp -o run -- python bench.py $B > $OUT/dp_traced.json 2> $OUT/dp_traced.err || { echo traced failed; tail -20 $OUT/dp_traced.err; exit 1; }
echo done
