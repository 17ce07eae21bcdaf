set -o pipefail
OUT=gpurun_out/r04_j7; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread --ignore=tests/test_gpu_fullsize.py > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
echo done
