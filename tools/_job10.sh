set -o pipefail
OUT=gpurun_out/r04_j10; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_smallk.py tests/test_gpu_res64pp.py tests/test_gpu_ops_r2.py tests/test_gpu_fcdensenet.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_new.log 2>&1 || { tail -40 $OUT/pytest_new.log; exit 1; }
tail -2 $OUT/pytest_new.log
BENCH_ARGS="--model fcdensenet" bash tools/ab_bench.sh r04_j10/ab "" "--option res16c_bh=8" "--option res16_dma=0" "--option res16c_bh=2" || exit 1
P2="--steps 4 --warmup 2 --no-cpu-baseline --no-traffic --no-miou --no-pipeline --no-extra --no-inference --no-dp-probe"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- python bench.py $P2 --model fcdensenet > $OUT/prof_c3.json 2> $OUT/prof_c3.err || { tail -30 $OUT/prof_c3.err; exit 1; }
echo done
