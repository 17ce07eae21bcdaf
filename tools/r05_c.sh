#!/bin/bash
# conv_halo2s: parity vs conv_halo2, kernel A/B, C2 step A/B
set -o pipefail
OUT=gpurun_out/${1:-r05_c}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_halo2s.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python tools/kbench.py conv3_2:fwd conv4_2:fwd conv4_1:fwd conv5_1:fwd conv3_2:dgrad conv4_2:dgrad conv4_1:dgrad --opts 'halo2_1p=0' --opts 'halo2_1p=1' --reps 20 --rounds 5 > $OUT/kbench.txt 2>&1 || { echo kbench failed; tail -20 $OUT/kbench.txt; exit 1; }
cat $OUT/kbench.txt
B="--no-extra --no-traffic --no-cpu-baseline --no-pipeline --no-inference --no-miou --no-dp-probe"
for o in 1 0 1 0; do
  timeout -k 10 300 python bench.py $B --option halo2_1p=$o > $OUT/bench_$o.json 2> $OUT/bench_$o.err || { echo bench failed; tail -20 $OUT/bench_$o.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_$o.json')); print('halo2_1p=$o', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline'].get('alone',{}).get('avg_launch_ms'))"
done
