set -o pipefail
OUT=gpurun_out/r04_j17; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_smallk.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_new.log 2>&1 || { tail -40 $OUT/pytest_new.log; exit 1; }
tail -2 $OUT/pytest_new.log
timeout -k 10 300 python -u tools/dense_kbench.py copy:384:1248:256 smallk:384:1248:256 smallk:384:1248:256:nm > $OUT/dense_kbench.txt 2>&1 || { tail -30 $OUT/dense_kbench.txt; exit 1; }
grep -v "^round" $OUT/dense_kbench.txt
SEG_DIAG_LIB=1 timeout -k 10 300 python -u tools/dense_kbench.py smallk:384:1248:256 --opts smallk_abl=0 --opts smallk_abl=1 --opts smallk_abl=2 --opts smallk_abl=3 > $OUT/dense_kbench_abl.txt 2>&1 || { tail -30 $OUT/dense_kbench_abl.txt; exit 1; }
grep -v "^round" $OUT/dense_kbench_abl.txt
BENCH_ARGS="--model fcdensenet" bash tools/ab_bench.sh r04_j17/ab3 "" || exit 1
echo done
