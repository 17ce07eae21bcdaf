set -o pipefail
OUT=gpurun_out/r04_j18; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
SKIP_TESTS=1 bash tools/gpu_round.sh r04_j18/round || exit 1
echo done
