export TMPDIR=/tmp
mkdir -p gpurun_out/r01d
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r01d/pytest.log 2>&1; rc=$?; tail -4 gpurun_out/r01d/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python bench.py --kernel-table --no-traffic --no-cpu-baseline > gpurun_out/r01d/bench.json 2> gpurun_out/r01d/kt.txt && cat gpurun_out/r01d/bench.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01d/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-traffic > /dev/null 2> gpurun_out/r01d/prof.err
