#!/bin/bash
# 8-channel resize kernels: bit-exact vs the per-element kernels, DeepLab parity, the C5 line twice
set -o pipefail
OUT=gpurun_out/r05_resize; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_deeplab.py tests/test_gpu_eval.py tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread -k "resize or deeplab or eval or golden or DeepLab" > $OUT/pytest.txt 2>&1 || { echo tests failed; tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
P="--no-cpu-baseline --no-traffic --no-miou --no-pipeline --no-extra --no-dp-probe --no-inference"
for i in 1 2; do
timeout -k 10 300 python bench.py --model deeplab $P > $OUT/c5_$i.json 2> $OUT/c5_$i.err || { echo bench failed; tail -20 $OUT/c5_$i.err; exit 1; }
grep -h '^{' $OUT/c5_$i.json | cut -c1-110
done
echo done
