export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "adam_fused" -x -q --timeout 120 --timeout-method thread > /tmp/pf.log 2>&1; rc=$?; tail -2 /tmp/pf.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" /tmp/pf.log | head; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_fcn.py -x -q --timeout 120 --timeout-method thread > /tmp/pf2.log 2>&1; rc=$?; tail -2 /tmp/pf2.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" /tmp/pf2.log | head; exit 1; }
for a in "--no-fuse-adam" ""; do
  timeout -k 10 200 python bench.py $a --kernel-table --no-traffic --no-cpu-baseline > /tmp/b.json 2> /tmp/kt.txt || exit 1
  echo "== $a: $(python -c "import json;print(json.load(open('/tmp/b.json'))['value'])")"; grep "op=2" /tmp/kt.txt | grep tn3
done
