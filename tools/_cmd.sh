#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/s2h; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "bwd_filter" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python tools/wg_probe.py "wgrad_la=1" "wgrad_la=3" > $OUT/wg.txt 2>&1 || { tail -20 $OUT/wg.txt; exit 1; }
cat $OUT/wg.txt
for opt in "" "wgrad_la=1" ""; do
  SEG_OPTIONS="$opt" timeout -k 10 200 python bench.py --no-traffic --no-cpu-baseline --no-miou --no-pipeline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "$opt $(python -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'])")"
done
