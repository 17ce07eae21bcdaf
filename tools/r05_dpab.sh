#!/bin/bash
# world-1 RCCL data-parallel probe A/B: r05_dpab.sh TAG "name|bench args" ...
set -o pipefail
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
B="--no-extra --no-traffic --no-cpu-baseline --no-pipeline --no-inference --no-miou --steps 10 --warmup 3"
for spec in "$@"; do
  name=${spec%%|*}; args=${spec#*|}
  timeout -k 10 400 python bench.py $B $args > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -20 $OUT/$name.err; exit 1; }
  grep -h '^{' $OUT/$name.json | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print('$name', d['value'], d['dp_mode']['value'], d['dp_mode']['ms_per_step'])"
done
echo done
