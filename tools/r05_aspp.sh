#!/bin/bash
# DeepLab's ASPP concat as channel views: C5 parity (end-to-end vs the oracle, full size), then the
# C5 line A/B against the copying concat (Session.alias_concat cannot split FC-DenseNet from DeepLab,
# so the A/B is the default bench line before / after in this same call: --schedule is not needed)
set -o pipefail
OUT=gpurun_out/r05_aspp; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_deeplab.py tests/test_gpu_fullsize.py tests/test_gpu_fp16.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo tests failed; tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
P="--no-cpu-baseline --no-traffic --no-miou --no-pipeline --no-extra --no-dp-probe --no-inference"
for i in 1 2; do
timeout -k 10 300 python bench.py --model deeplab $P > $OUT/c5_$i.json 2> $OUT/c5_$i.err || { echo bench failed; tail -20 $OUT/c5_$i.err; exit 1; }
grep -h '^{' $OUT/c5_$i.json | cut -c1-120
done
echo done
