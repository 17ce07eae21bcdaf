#!/bin/bash
# CU-masked fused conv6/conv7 update: correctness (RCCL schedule test), C2 A/B, trace
set -o pipefail
OUT=gpurun_out/${1:-r05_d}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp_rccl.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
B="--no-extra --no-traffic --no-cpu-baseline --no-pipeline --no-inference --no-miou --no-dp-probe"
for s in "fused_cu_pct=0" "fused_cu_pct=50" "fused_cu_pct=25" "fused_cu_pct=50 fused_cu_contig=1" "fused_cu_pct=75" "fused_cu_pct=50 fused_delay=0" "fused_cu_pct=0"; do
  args=""; for kv in $s; do args="$args --schedule $kv"; done
  tag=$(echo $s | tr ' =' '__')
  timeout -k 10 300 python bench.py $B $args > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { echo bench failed; tail -20 $OUT/b_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b_$tag.json')); r=d['roofline']; print('$s', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['all_events_avg_launch_ms'], r.get('alone',{}).get('avg_launch_ms'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof50 -o run -- python bench.py --steps 10 --warmup 3 $B --schedule fused_cu_pct=50 > $OUT/prof50.json 2> $OUT/prof50.err || { echo rocprof failed; tail -20 $OUT/prof50.err; exit 1; }
echo done
