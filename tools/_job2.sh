set -o pipefail
OUT=gpurun_out/r04_j2; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests/test_gpu_fullsize.py -x -v -s -k "c3 or c2_end" --timeout 1000 --timeout-method thread > $OUT/pytest_full.log 2>&1 || { tail -60 $OUT/pytest_full.log; exit 1; }
tail -3 $OUT/pytest_full.log
timeout -k 10 200 python tools/shadow_probe.py conv4_2:fwd conv3_2:dgrad conv4_2:wgrad conv2_2:fwd conv1_2:dgrad > $OUT/shadow.txt 2>&1 || { tail -20 $OUT/shadow.txt; exit 1; }
cat $OUT/shadow.txt
echo done
