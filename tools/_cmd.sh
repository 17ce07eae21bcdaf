export TMPDIR=/tmp
mkdir -p gpurun_out/r01e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r01e/pytest.log 2>&1; rc=$?; tail -4 gpurun_out/r01e/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r01e/pytest.log | head -20; exit 1; }
timeout -k 10 200 python bench.py --kernel-table --no-traffic --no-cpu-baseline > gpurun_out/r01e/bench.json 2> gpurun_out/r01e/kt.txt && cat gpurun_out/r01e/bench.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01e/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-traffic > /dev/null 2> gpurun_out/r01e/prof.err
