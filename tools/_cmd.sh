export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_eval.py -x -q --timeout 120 --timeout-method thread > /tmp/pe.log 2>&1; rc=$?; tail -2 /tmp/pe.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" /tmp/pe.log | head -20; exit 1; }
