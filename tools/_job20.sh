set -o pipefail
OUT=gpurun_out/r04_j20; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops_r2.py tests/test_gpu_bn2.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_new.log 2>&1 || { tail -40 $OUT/pytest_new.log; exit 1; }
tail -2 $OUT/pytest_new.log
timeout -k 10 300 python -u tools/dense_kbench.py fwdbn2:384:1248:128 fwdbn2:384:1248:48 fwdbn2:192:624:144 --opts s1x1_st=0 --opts s1x1_st=1 > $OUT/dense_kbench.txt 2>&1 || { tail -30 $OUT/dense_kbench.txt; exit 1; }
grep -v "^round" $OUT/dense_kbench.txt
BENCH_ARGS="--model fcdensenet" bash tools/ab_bench.sh r04_j20/ab "" "--option s1x1_st=1" || exit 1
echo done
