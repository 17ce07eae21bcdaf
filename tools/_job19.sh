set -o pipefail
OUT=gpurun_out/r04_j19; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops_r2.py tests/test_gpu_fcdensenet.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_new.log 2>&1 || { tail -40 $OUT/pytest_new.log; exit 1; }
tail -2 $OUT/pytest_new.log
timeout -k 10 300 python -u tools/dense_kbench.py bn1x1:384:1248:128 bn1x1:384:1248:48 bn1x1:192:624:160 --opts bn1x1s_st=1 --opts bn1x1s_st=0 > $OUT/dense_kbench.txt 2>&1 || { tail -30 $OUT/dense_kbench.txt; exit 1; }
grep -v "^round" $OUT/dense_kbench.txt
BENCH_ARGS="--model fcdensenet" bash tools/ab_bench.sh r04_j19/ab "" "--option bn1x1s_st=0" || exit 1
echo done
