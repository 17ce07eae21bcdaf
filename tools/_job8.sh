set -o pipefail
OUT=gpurun_out/r04_j8; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_smallk.py tests/test_gpu_bn2.py tests/test_gpu_fcdensenet.py tests/test_gpu_res64pp.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_new.log 2>&1 || { tail -40 $OUT/pytest_new.log; exit 1; }
tail -2 $OUT/pytest_new.log
P="--steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-miou --no-pipeline --no-extra --no-inference --no-dp-probe"
timeout -k 10 300 python bench.py $P --model fcdensenet > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -30 $OUT/bench_c3.err; exit 1; }
cat $OUT/bench_c3.json
timeout -k 10 300 python bench.py $P > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -30 $OUT/bench_c2.err; exit 1; }
cat $OUT/bench_c2.json
P2="--steps 4 --warmup 2 --no-cpu-baseline --no-traffic --no-miou --no-pipeline --no-extra --no-inference --no-dp-probe"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- python bench.py $P2 --model fcdensenet > $OUT/prof_c3.json 2> $OUT/prof_c3.err || { tail -30 $OUT/prof_c3.err; exit 1; }
echo done
