#!/bin/bash
# scratch command for one gpurun call (not product; see tools/gpu_round.sh for the full pass)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-scratch}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_fp16.py > $OUT/t.log 2>&1 || { tail -60 $OUT/t.log; exit 1; }
tail -3 $OUT/t.log
timeout -k 10 200 python bench.py --model deeplab --steps 5 --warmup 3 --no-traffic --no-miou --no-cpu-baseline --no-pipeline --kernel-table > $OUT/c5.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/c5.json'));print('c5', d['dtype'], d['value'], d['ms_per_step'], d.get('loss_scaling'))"
grep GROUP $OUT/c5.err
