set -o pipefail
OUT=gpurun_out/r04_j5; mkdir -p $OUT; export TMPDIR=/tmp
P="--steps 4 --warmup 2 --no-cpu-baseline --no-traffic --no-miou --no-pipeline --no-extra --no-inference --no-dp-probe"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3 -o run -- python bench.py $P --model fcdensenet > $OUT/prof_c3.json 2> $OUT/prof_c3.err || { tail -30 $OUT/prof_c3.err; exit 1; }
cat $OUT/prof_c3.json
timeout -k 10 1000 python -u -m pytest tests/test_gpu_fullsize.py -x -v -s -k "c3" --timeout 950 --timeout-method thread > $OUT/pytest_c3.log 2>&1 || { grep -E "GRAD|PASS|FAIL|Error|assert" $OUT/pytest_c3.log | tail -40; exit 1; }
grep -E "GRAD|passed|failed|C3 image" $OUT/pytest_c3.log | tail -60
echo done
