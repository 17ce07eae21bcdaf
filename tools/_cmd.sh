#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/s2f; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_ops.py -k "eval or gen_test or adam" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for opt in "" "halo2_n128=1" "tn3_mfast=1" "tn3_stagger_us=0" "tn3_half=0" "wgrad_nbias=4" "halo_phases=4"; do
  SEG_OPTIONS="$opt" timeout -k 10 200 python bench.py --no-traffic --no-cpu-baseline --no-miou --no-pipeline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "$opt $(python -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'])")"
done
