set -o pipefail
OUT=gpurun_out/r04_j3; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_fullsize.py -x -v -s -k "c3 or c2_end" --timeout 950 --timeout-method thread > $OUT/pytest_c3.log 2>&1 || { grep -E "GRAD|PASS|FAIL|Error|assert" $OUT/pytest_c3.log | tail -40; exit 1; }
grep -E "GRAD|passed|failed" $OUT/pytest_c3.log | tail -60
echo done
