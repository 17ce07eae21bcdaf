#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/s2a; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_checkpoint.py -k "prepare_input or checkpoint" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python bench.py --kernel-table --no-traffic --no-cpu-baseline --no-miou > $OUT/bench.json 2> $OUT/kt.txt || { tail -30 $OUT/kt.txt; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-traffic --no-miou > $OUT/prof_bench.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
python tools/timeline.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) > $OUT/timeline.txt
head -40 $OUT/timeline.txt
