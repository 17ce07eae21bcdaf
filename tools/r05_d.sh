#!/bin/bash
# CU-masked fused conv6/conv7 update (C2 A/B), grouped dropout hash (parity), persistent-grid fills (C3 A/B)
set -o pipefail
OUT=gpurun_out/${1:-r05_d}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp_rccl.py tests/test_gpu_dropout_fusion.py tests/test_gpu_dropout_flat.py tests/test_gpu_ops_r2.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
B="--no-extra --no-traffic --no-cpu-baseline --no-pipeline --no-inference --no-miou --no-dp-probe"
run() {  # tag, args...
  tag=$1; shift
  timeout -k 10 300 python bench.py $B "$@" > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { echo bench $tag failed; tail -20 $OUT/b_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b_$tag.json')); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['all_events_avg_launch_ms'], r.get('alone',{}).get('avg_launch_ms'))"
}
run c2_base
run c2_cu50 --schedule fused_cu_pct=50
run c2_cu25 --schedule fused_cu_pct=25
run c2_cu50c --schedule fused_cu_pct=50 --schedule fused_cu_contig=1
run c2_cu75 --schedule fused_cu_pct=75
run c2_cu50d0 --schedule fused_cu_pct=50 --schedule fused_delay=0
run c2_res2 --option res64_fill=2
run c2_base2
run c3_base --model fcdensenet --steps 8 --warmup 3
run c3_bn2 --model fcdensenet --steps 8 --warmup 3 --option bn1x1s_fill=2
run c3_bn2s2 --model fcdensenet --steps 8 --warmup 3 --option bn1x1s_fill=2 --option s1x1_fill=2
run c3_bn4s2 --model fcdensenet --steps 8 --warmup 3 --option bn1x1s_fill=4 --option s1x1_fill=2
run c3_wf50 --model fcdensenet --steps 8 --warmup 3 --option wgrad_fill16=50
run c3_base2 --model fcdensenet --steps 8 --warmup 3
echo done
