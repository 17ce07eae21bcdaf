set -o pipefail
OUT=gpurun_out/r04_j4; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_res64pp.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_res64pp.log 2>&1 || { tail -40 $OUT/pytest_res64pp.log; exit 1; }
tail -2 $OUT/pytest_res64pp.log
P="--steps 10 --warmup 3 --no-cpu-baseline --no-traffic --no-miou --no-pipeline --no-extra --no-inference --no-dp-probe"
timeout -k 10 300 python bench.py $P --model fcdensenet --kernel-table > $OUT/bench_c3.json 2> $OUT/bench_c3_table.txt || { tail -30 $OUT/bench_c3_table.txt; exit 1; }
cat $OUT/bench_c3.json
timeout -k 10 1000 python -u -m pytest tests/test_gpu_fullsize.py -x -v -s -k "c3_layer or c3_grad" --timeout 950 --timeout-method thread > $OUT/pytest_c3.log 2>&1 || { grep -E "GRAD|PASS|FAIL|Error|assert" $OUT/pytest_c3.log | tail -40; exit 1; }
grep -E "GRAD|passed|failed" $OUT/pytest_c3.log | tail -60
echo done
