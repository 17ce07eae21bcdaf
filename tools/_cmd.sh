#!/bin/bash
# scratch command for one gpurun call (not product; see tools/gpu_round.sh for the full pass)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-scratch}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train_api.py tests/test_gpu_dp.py tests/test_gpu_fullsize.py > $OUT/t.log 2>&1 || { tail -60 $OUT/t.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $OUT/t.log | tail -30
