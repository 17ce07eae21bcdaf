#!/bin/bash
# A/B bench runs in one call: r05_ab.sh TAG "name|bench args" ... (alternating order is the caller's)
# optional: PRE_TEST=<pytest node id> runs first
set -o pipefail
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
if [ -n "$PRE_TEST" ]; then
  timeout -k 10 800 python -u -m pytest $PRE_TEST -x -q --timeout 300 --timeout-method thread > $OUT/pre_test.log 2>&1 || { echo pre-test failed; tail -30 $OUT/pre_test.log; exit 1; }
  tail -1 $OUT/pre_test.log
fi
B="--no-extra --no-traffic --no-cpu-baseline --no-pipeline --no-inference --no-miou --no-dp-probe"
for spec in "$@"; do
  name=${spec%%|*}; args=${spec#*|}
  timeout -k 10 300 python bench.py $B $args > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -20 $OUT/$name.err; exit 1; }
  python -c "
import json,sys
for l in open('$OUT/$name.json'):
    if l.startswith('{'):
        d=json.loads(l); r=d.get('roofline',{}); print('$name', d['value'], d['ms_per_step'], r.get('kernel'), r.get('frac'))"
done
echo done
