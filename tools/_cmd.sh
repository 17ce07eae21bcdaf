#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/s2q; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fcdensenet.py tests/test_gpu_deeplab.py -k "bn or fcdense or deeplab or relu or concat" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log


timeout -k 10 400 python bench.py --model fcdensenet --no-traffic --no-miou --no-cpu-baseline --no-pipeline > $OUT/c3.json 2> $OUT/c3.err || { tail -20 $OUT/c3.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/c3.json'));print(d['value'], d['ms_per_step'])"
