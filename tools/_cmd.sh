#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/s2d; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_augment.py tests/test_png_decode.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python bench.py --no-traffic --no-cpu-baseline --no-miou > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
