export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_deeplab.py -x -q --timeout 200 --timeout-method thread > /tmp/pd.log 2>&1; rc=$?; tail -2 /tmp/pd.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" /tmp/pd.log | head -20; exit 1; }
timeout -k 10 300 python bench.py --model deeplab --steps 10 --warmup 3 --kernel-table --no-traffic --no-cpu-baseline > /tmp/b.json 2> /tmp/kt.txt; rc=$?; cat /tmp/b.json; [ $rc -eq 0 ] || { tail -20 /tmp/kt.txt; exit 1; }
grep GROUP /tmp/kt.txt
