#!/bin/bash
# Focused GPU pass: named test files, smoke, bench, single-launch timings.
# usage: tools/gpu_quick.sh TAG "tests... [-k 'expr']" "kbench specs" [bench args...]  (TESTS is eval'd)
set -o pipefail
TAG=$1; TESTS=$2; KB=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  eval timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
  tail -3 $OUT/pytest.log
fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 400 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
if [ -n "$KB" ]; then
  timeout -k 10 300 python tools/kbench.py $KB > $OUT/kbench.txt 2>&1 || { echo kbench failed; tail -30 $OUT/kbench.txt; exit 1; }
  cat $OUT/kbench.txt
fi
echo done
