set -o pipefail
OUT=gpurun_out/r04_j1; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp_rccl.py tests/test_gpu_dp.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_dp.log 2>&1 || { tail -40 $OUT/pytest_dp.log; exit 1; }
tail -3 $OUT/pytest_dp.log
timeout -k 10 1500 python -u -m pytest tests/test_gpu_fullsize.py -x -v -s -k "c3 or c2_end" --timeout 1200 --timeout-method thread > $OUT/pytest_full.log 2>&1 || { tail -60 $OUT/pytest_full.log; exit 1; }
tail -3 $OUT/pytest_full.log
P="--steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-miou --no-pipeline --no-extra --no-inference"
timeout -k 10 400 python bench.py $P > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo done
