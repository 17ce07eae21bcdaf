#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/s2i; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -k "conv2d" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for opt in "" ""; do
  SEG_OPTIONS="$opt" timeout -k 10 200 python bench.py --no-traffic --no-cpu-baseline --no-miou --no-pipeline --kernel-table > $OUT/b.json 2> $OUT/kt.txt || { tail -20 $OUT/kt.txt; exit 1; }
  echo "$opt $(python -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'])")"
done
grep GROUP $OUT/kt.txt
