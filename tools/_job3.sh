set -o pipefail
OUT=gpurun_out/r04_j3; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_res64pp.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_res64pp.log 2>&1 || { tail -40 $OUT/pytest_res64pp.log; exit 1; }
tail -2 $OUT/pytest_res64pp.log
timeout -k 10 200 python tools/kbench.py conv1_2:fwdpool conv1_2:dgrad conv1_2:fwd --opts 'res64_pp=1' --opts 'res64_pp=0' --rounds 5 --reps 10 > $OUT/kbench_res64.txt 2>&1 || { tail -20 $OUT/kbench_res64.txt; exit 1; }
cat $OUT/kbench_res64.txt
bash tools/ab_bench.sh r04_j3/ab "" "--option res64_pp=0" || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -v -s -k "c3 or c2_end" --timeout 850 --timeout-method thread > $OUT/pytest_c3.log 2>&1 || { grep -E "GRAD|PASS|FAIL|Error|assert" $OUT/pytest_c3.log | tail -40; exit 1; }
grep -E "GRAD|passed|failed" $OUT/pytest_c3.log | tail -60
echo done
