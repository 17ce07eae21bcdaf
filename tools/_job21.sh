set -o pipefail
OUT=gpurun_out/r04_j21; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops_r2.py tests/test_gpu_bn2.py tests/test_gpu_fcdensenet.py tests/test_gpu_smallk.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_new.log 2>&1 || { tail -40 $OUT/pytest_new.log; exit 1; }
tail -2 $OUT/pytest_new.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json | cut -c1-300
P="--steps 10 --warmup 3 --no-cpu-baseline --no-traffic --no-miou --no-pipeline --no-extra --no-dp-probe --no-inference"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_fcdensenet -o run -- python bench.py $P --model fcdensenet > $OUT/prof_fcdensenet.json 2> $OUT/prof_fcdensenet.err || { tail -20 $OUT/prof_fcdensenet.err; exit 1; }
echo done
