#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprof kernel stats (C2 alone,
# then the C3 / C5 side configs), HBM PMC passes inside bench.py.
# usage: tools/gpu_round.sh TAG [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -3 $OUT/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 400 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
P="--steps 10 --warmup 3 --no-cpu-baseline --no-traffic --no-miou --no-pipeline --no-extra --no-dp-probe --no-inference"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py $P "$@" > $OUT/prof_bench.json 2> $OUT/prof.err || { echo rocprof failed; tail -20 $OUT/prof.err; exit 1; }
for m in fcdensenet deeplab; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$m -o run -- python bench.py $P --model $m > $OUT/prof_$m.json 2> $OUT/prof_$m.err || { echo rocprof $m failed; tail -20 $OUT/prof_$m.err; exit 1; }
done
echo done
