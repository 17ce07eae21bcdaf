#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/s3d; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_dropout_fusion.py -k "dropout or conv" > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
timeout -k 10 300 python bench.py --model fcdensenet --steps 10 --warmup 3 --no-traffic --no-miou --no-cpu-baseline --no-pipeline > $OUT/c3.json 2> $OUT/c3.err || { tail -20 $OUT/c3.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/c3.json'));print('c3', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --model fcdensenet --steps 2 --warmup 2 --no-traffic --no-miou --no-cpu-baseline --no-pipeline --kernel-table > $OUT/kt.json 2> $OUT/kt.err || exit 1
grep "KERNEL igemm_nt2" $OUT/kt.err | grep "384x1248" | grep "op=0" | sed 's/.*ms= *\([0-9.]*\).*C=\([0-9]*\) K.*/\2:\1/' | tr '\n' ' '
