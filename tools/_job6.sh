set -o pipefail
OUT=gpurun_out/r04_j6; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 200 python tools/host_probe.py --model fcn > $OUT/host_fcn.txt 2>&1 || { tail -30 $OUT/host_fcn.txt; exit 1; }
head -40 $OUT/host_fcn.txt
timeout -k 10 300 python tools/host_probe.py --model fcdensenet > $OUT/host_c3.txt 2>&1 || { tail -30 $OUT/host_c3.txt; exit 1; }
head -40 $OUT/host_c3.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_bn2.py tests/test_gpu_fcdensenet.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_bn2.log 2>&1 || { tail -40 $OUT/pytest_bn2.log; exit 1; }
tail -2 $OUT/pytest_bn2.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -v -s -k "c3_layer or c3_grad or c3_end" --timeout 850 --timeout-method thread > $OUT/pytest_c3.log 2>&1 || { grep -E "GRAD|PASS|FAIL|Error|assert" $OUT/pytest_c3.log | tail -40; exit 1; }
grep -E "GRAD|passed|failed|C3 image" $OUT/pytest_c3.log | tail -40
echo done
