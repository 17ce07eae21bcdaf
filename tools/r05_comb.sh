#!/bin/bash
# igemm_nt3's in-launch 2-way split-K combine: bit-exact vs the reducer, the split-K parity
# suites, the default bench line, and a traced C2 run (step composition with the reducers gone)
set -o pipefail
OUT=gpurun_out/r05_comb; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_nt3_combine.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_comb.txt 2>&1 || { echo combine tests failed; tail -30 $OUT/pytest_comb.txt; exit 1; }
grep -c PASSED $OUT/pytest_comb.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_ops_r2.py tests/test_gpu_fullsize.py tests/test_gpu_fcn.py tests/test_gpu_golden.py tests/test_gpu_dropout_fusion.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo tests failed; tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
timeout -k 10 700 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
grep -h '^{' $OUT/bench.json | cut -c1-140
P="--no-cpu-baseline --no-traffic --no-miou --no-pipeline --no-extra --no-dp-probe --no-inference"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_fcn -o run -- python bench.py --steps 10 --warmup 3 $P > $OUT/prof_fcn.json 2> $OUT/prof_fcn.err || { echo rocprof failed; tail -20 $OUT/prof_fcn.err; exit 1; }
grep -h "splitk_reduce_nt\|igemm_nt3" $OUT/prof_fcn/run_kernel_stats.csv | cut -c1-120
echo done
