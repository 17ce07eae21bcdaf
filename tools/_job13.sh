set -o pipefail
OUT=gpurun_out/r04_j13; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_smallk.py tests/test_gpu_ops_r2.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_new.log 2>&1 || { tail -40 $OUT/pytest_new.log; exit 1; }
tail -2 $OUT/pytest_new.log
timeout -k 10 400 python -u tools/dense_kbench.py copy:384:1248:256 smallk:384:1248:256 smallk:384:1248:256:nm bn1x1:384:1248:128 bn1x1:12:39:414 bn3x3:384:1248 bn3x3:384:1248:nd fwdbn2:384:1248:128 fwdbn2:384:1248:128:nd fwdbn2:384:1248:48 fwdbn2:384:1248:48:nd grow:384:1248 grow:384:1248:nd > $OUT/dense_kbench.txt 2>&1 || { tail -30 $OUT/dense_kbench.txt; exit 1; }
grep -v "^round" $OUT/dense_kbench.txt
BENCH_ARGS="--model fcdensenet" bash tools/ab_bench.sh r04_j13/ab "" || exit 1
echo done
