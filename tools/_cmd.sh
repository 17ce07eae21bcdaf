#!/bin/bash
# scratch command for one gpurun call (not product; see tools/gpu_round.sh for the full pass)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-scratch}; mkdir -p $OUT
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "wgrad or filter" > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
B="python bench.py --steps 20 --warmup 5 --no-traffic --no-miou --no-cpu-baseline --no-pipeline --no-extra"
for o in tn_reduce_sl=16 tn_reduce_sl=1 tn_reduce_sl=4; do
  timeout -k 10 200 $B --option $o > $OUT/c2_$o.json 2> $OUT/c2_$o.err || { tail -20 $OUT/c2_$o.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c2_$o.json'));print('$o', d['value'], d['ms_per_step'])"
done
for m in fcdensenet; do
  timeout -k 10 200 $B --model $m --steps 10 --warmup 3 --option tn_reduce_sl=16 > $OUT/$m.json 2> $OUT/$m.err || { tail -20 $OUT/$m.err; exit 1; }
  timeout -k 10 200 $B --model $m --steps 10 --warmup 3 --option tn_reduce_sl=1 > $OUT/${m}1.json 2> $OUT/${m}1.err || { tail -20 $OUT/${m}1.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$m.json'));e=json.load(open('$OUT/${m}1.json'));print('$m sl16', d['value'], 'sl1', e['value'])"
done
