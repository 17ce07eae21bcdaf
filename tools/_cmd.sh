#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/s2l; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "nt4" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python tools/gemm_probe.py > $OUT/gp.txt 2>&1 || { tail -20 $OUT/gp.txt; exit 1; }
cat $OUT/gp.txt
