#!/bin/bash
# rocprofv3 kernel trace of C3 (FC-DenseNet) bench steps: r05_c3trace.sh TAG [extra bench args]
set -o pipefail
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
P="--no-cpu-baseline --no-traffic --no-miou --no-pipeline --no-extra --no-dp-probe --no-inference"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- python bench.py --model fcdensenet --steps 5 --warmup 3 $P "$@" > $OUT/prof_c3.json 2> $OUT/prof_c3.err || { echo rocprof c3 failed; tail -20 $OUT/prof_c3.err; exit 1; }
echo c3 trace done
