#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/s2j; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_golden.py tests/test_gpu_fcn.py -k "adam or golden or fcn" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
PROBE_ABL=0 timeout -k 10 200 python tools/adam_probe.py > $OUT/ap.txt 2>&1 || { tail -20 $OUT/ap.txt; exit 1; }
SEG_OPTIONS=adam_tr_fused=1 PROBE_ABL=0 timeout -k 10 200 python tools/adam_probe.py >> $OUT/ap.txt 2>&1 || { tail -20 $OUT/ap.txt; exit 1; }
grep adam $OUT/ap.txt
for opt in "" "adam_tr_fused=1" ""; do
  SEG_OPTIONS="$opt" timeout -k 10 200 python bench.py --no-traffic --no-cpu-baseline --no-miou --no-pipeline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "$opt $(python -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'])")"
done
