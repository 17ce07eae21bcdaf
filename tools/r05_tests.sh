#!/bin/bash
# full GPU suite + smoke, then per-launch kernel tables of C2 and C3
set -o pipefail
OUT=gpurun_out/${1:-r05_t}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 960 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
B="--no-extra --no-traffic --no-cpu-baseline --no-pipeline --no-inference --no-miou --no-dp-probe --kernel-table"
timeout -k 10 200 python bench.py $B > $OUT/kt_c2.json 2> $OUT/kt_c2.err || { echo kt c2 failed; tail -5 $OUT/kt_c2.err; exit 1; }
timeout -k 10 200 python bench.py $B --model fcdensenet --steps 5 --warmup 3 > $OUT/kt_c3.json 2> $OUT/kt_c3.err || { echo kt c3 failed; tail -5 $OUT/kt_c3.err; exit 1; }
grep -h '^{' $OUT/kt_c2.json $OUT/kt_c3.json | cut -c1-200
echo done
