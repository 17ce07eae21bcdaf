#!/bin/bash
# scratch command for one gpurun call (not product; see tools/gpu_round.sh for the full pass)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-scratch}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "conv2d" > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py -k "c3" > $OUT/t2.log 2>&1 || { tail -30 $OUT/t2.log; exit 1; }
tail -1 $OUT/t2.log
B="python bench.py --steps 10 --warmup 3 --no-traffic --no-miou --no-cpu-baseline --no-pipeline --no-extra"
run() { n=$1; shift; timeout -k 10 200 $B "$@" > $OUT/$n.json 2> $OUT/$n.err || { tail -20 $OUT/$n.err; exit 1; }; python -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', d['value'], d['ms_per_step'])"; }
run c3 --model fcdensenet
run c3_nt2 --model fcdensenet --option res16c=0
