#!/bin/bash
# end of round 5: full GPU suite + smoke on the final tree, then the default bench line
set -o pipefail
OUT=gpurun_out/r05_end; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; cat $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
timeout -k 10 700 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
python -c "
import json; d=json.loads([l for l in open('$OUT/bench.json') if l.startswith('{')][0])
print('C2', d['value'], d['roofline']['frac'], 'C3', d['c3_fcdensenet']['value'], 'C5', d['c5_deeplab']['value'], 'dp', d['dp_mode']['value'], 'cpu', d['cpu_baseline']['value'])"
echo done
