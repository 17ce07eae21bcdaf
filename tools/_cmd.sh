#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/s3l; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_fcdensenet.py tests/test_gpu_golden.py > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
timeout -k 10 300 python bench.py --model fcdensenet --steps 10 --warmup 3 --no-traffic --no-miou --no-cpu-baseline --no-pipeline > $OUT/c3.json 2> $OUT/c3.err || { tail -20 $OUT/c3.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/c3.json'));print('c3', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --model deeplab --steps 5 --warmup 2 --no-traffic --no-miou --no-cpu-baseline --no-pipeline > $OUT/c5.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/c5.json'));print('c5', d['value'], d['ms_per_step'])"
