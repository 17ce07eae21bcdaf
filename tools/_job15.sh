set -o pipefail
OUT=gpurun_out/r04_j15; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_smallk.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_new.log 2>&1 || { tail -40 $OUT/pytest_new.log; exit 1; }
tail -2 $OUT/pytest_new.log
timeout -k 10 300 python -u tools/dense_kbench.py copy:384:1248:256 smallk:384:1248:256 smallk:384:1248:256:nm > $OUT/dense_kbench.txt 2>&1 || { tail -30 $OUT/dense_kbench.txt; exit 1; }
grep -v "^round" $OUT/dense_kbench.txt
BENCH_ARGS="--model fcdensenet" bash tools/ab_bench.sh r04_j15/ab3 "" || exit 1
bash tools/ab_bench.sh r04_j15/ab2 "" "--option adam_tr_fused=1" "--schedule fused_delay=4" "--schedule main_wgrad=0" "--option tn_fill=3" || exit 1
echo done
