#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r05_g}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_dp_rccl.py tests/test_gpu_fcdensenet.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python tools/kbench.py conv6:wgrad conv7:wgrad conv6:wgrad_adam conv3_2:wgrad --reps 10 --rounds 3 > $OUT/kb.txt 2>&1 || { echo kbench failed; tail -20 $OUT/kb.txt; exit 1; }
cat $OUT/kb.txt
B="--no-extra --no-traffic --no-cpu-baseline --no-pipeline --no-inference --no-miou"
run() {  # tag, args...
  tag=$1; shift
  timeout -k 10 300 python bench.py $B "$@" > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { echo bench $tag failed; tail -20 $OUT/b_$tag.err; exit 1; }
  python -c "
import json
L=[l for l in open('$OUT/b_$tag.json') if l.startswith('{')][0]; d=json.loads(L); r=d['roofline']; dp=d.get('dp_mode') or {}
print('$tag', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], 'dp', dp.get('value'), dp.get('ms_per_step'))"
}
run c2a
run c2big --schedule overlap_big_mb=16
run c2b --no-dp-probe
run c3 --model fcdensenet --steps 8 --warmup 3
echo done
