#!/bin/bash
# BN(+ReLU) second output from splitk_reduce_nt (DeepLab's split igemm_nt3 ASPP convs): parity
# (bn2 bit-exact cases, C5 end to end, split-K NT suites, C3), the C5 line twice, the default line
set -o pipefail
OUT=gpurun_out/r05_bn2; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_bn2.py tests/test_gpu_deeplab.py tests/test_gpu_fullsize.py tests/test_gpu_fp16.py tests/test_gpu_ops.py tests/test_gpu_fcdensenet.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo tests failed; tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
P="--no-cpu-baseline --no-traffic --no-miou --no-pipeline --no-extra --no-dp-probe --no-inference"
for i in 1 2; do
timeout -k 10 300 python bench.py --model deeplab $P > $OUT/c5_$i.json 2> $OUT/c5_$i.err || { echo bench failed; tail -20 $OUT/c5_$i.err; exit 1; }
grep -h '^{' $OUT/c5_$i.json | cut -c1-110
done
timeout -k 10 700 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
python -c "
import json; d=json.loads([l for l in open('$OUT/bench.json') if l.startswith('{')][0])
print('C2', d['value'], 'C3', d['c3_fcdensenet']['value'], 'C5', d['c5_deeplab']['value'], 'dp', d['dp_mode']['value'], 'cpu', d['cpu_baseline']['value'])"
echo done
