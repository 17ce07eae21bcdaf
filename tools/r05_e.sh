#!/bin/bash
# reducer (8 loads in flight) A/B, DP overlap of the big layers' Adam, conv6 fused wgrad+Adam ablation
set -o pipefail
OUT=gpurun_out/${1:-r05_e}; mkdir -p $OUT; export TMPDIR=/tmp
B="--no-extra --no-traffic --no-cpu-baseline --no-pipeline --no-inference --no-miou"
run() {  # tag, args...
  tag=$1; shift
  timeout -k 10 300 python bench.py $B "$@" > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { echo bench $tag failed; tail -20 $OUT/b_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b_$tag.json')); r=d['roofline']; dp=d.get('dp_mode') or {}; print('$tag', d['value'], d['ms_per_step'], r['avg_launch_ms'], 'dp', dp.get('value'), dp.get('ms_per_step'))"
}
run base
run sl4 --option tn_reduce_sl=4 --no-dp-probe
run sl8 --option tn_reduce_sl=8 --no-dp-probe
run big16 --schedule overlap_big_mb=16
run base2
SEG_DIAG_LIB=1 timeout -k 10 300 python tools/kbench.py conv6:wgrad_adam conv6:wgrad conv7:wgrad_adam --opts 'tn3_adam_abl=0' --opts 'tn3_adam_abl=1' --opts 'tn3_adam_abl=2' --opts 'tn3_adam_abl=3' --opts 'tn3_adam_abl=12' --opts 'tn3_adam_abl=16' --reps 5 --rounds 3 > $OUT/kb_adam.txt 2>&1 || { echo kbench failed; tail -20 $OUT/kb_adam.txt; exit 1; }
cat $OUT/kb_adam.txt
echo done
