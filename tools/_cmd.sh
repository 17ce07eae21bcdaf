export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "begin_end" -x -q --timeout 120 --timeout-method thread > /tmp/p1.log 2>&1; rc=$?; tail -2 /tmp/p1.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" /tmp/p1.log | head -20; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > /tmp/pt.log 2>&1; rc=$?; tail -2 /tmp/pt.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" /tmp/pt.log | head -20; exit 1; }
for a in "" ; do
timeout -k 10 200 python bench.py --kernel-table --no-traffic --no-cpu-baseline --no-miou > /tmp/b.json 2> /tmp/kt.txt || exit 1
python -c "import json;print(json.load(open('/tmp/b.json'))['value'])"
done
