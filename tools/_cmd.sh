#!/bin/bash
# scratch command for one gpurun call (not product; see tools/gpu_round.sh for the full pass)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-scratch}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops_r2.py tests/test_gpu_deeplab.py tests/test_gpu_fullsize.py -k "deeplab or c5 or spatial or axpy" > $OUT/t.log 2>&1 || { tail -60 $OUT/t.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $OUT/t.log | tail -30
timeout -k 10 200 python bench.py --model deeplab --steps 5 --warmup 2 --no-traffic --no-miou --no-cpu-baseline --no-pipeline > $OUT/c5.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/c5.json'));print('c5', d['value'], d['ms_per_step'])"
