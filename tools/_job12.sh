set -o pipefail
OUT=gpurun_out/r04_j12; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/probe_bn.py > $OUT/probe_bn.txt 2>&1; cat $OUT/probe_bn.txt | grep -v amdgpu.ids
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops_r2.py tests/test_gpu_fcdensenet.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_new.log 2>&1 || { tail -40 $OUT/pytest_new.log; exit 1; }
tail -2 $OUT/pytest_new.log
timeout -k 10 400 python -u tools/dense_kbench.py bn1x1:384:1248:128 bn1x1:384:1248:48 bn1x1:192:624:160 bn1x1:12:39:414 bn3x3:384:1248 bn3x3:192:624 fwdbn2:384:1248:128 fwdbn2:384:1248:48 grow:384:1248 smallk:384:1248:256 --opts 'bn1x1s=1,nt2bn_bm=256,res16c_bh=4' --opts 'bn1x1s=0,nt2bn_bm=128,res16c_bh=8' --opts 'bn1x1s=0,nt2bn_bm=256,res16c_bh=4' > $OUT/dense_kbench.txt 2>&1 || { tail -30 $OUT/dense_kbench.txt; exit 1; }
grep -v "^round" $OUT/dense_kbench.txt
BENCH_ARGS="--model fcdensenet" bash tools/ab_bench.sh r04_j12/ab "" "--option bn1x1s=0" || exit 1
P2="--steps 4 --warmup 2 --no-cpu-baseline --no-traffic --no-miou --no-pipeline --no-extra --no-inference --no-dp-probe"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- python bench.py $P2 --model fcdensenet > $OUT/prof_c3.json 2> $OUT/prof_c3.err || { tail -30 $OUT/prof_c3.err; exit 1; }
echo done
