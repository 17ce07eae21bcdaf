set -o pipefail
OUT=gpurun_out/r04_j2; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 200 python tools/shadow_probe.py conv4_2:fwd conv3_2:dgrad conv4_2:wgrad conv2_2:fwd conv1_2:dgrad > $OUT/shadow.txt 2>&1 || { tail -20 $OUT/shadow.txt; exit 1; }
cat $OUT/shadow.txt
timeout -k 10 240 python tools/kbench.py conv5_1:fwd conv5_1:dgrad conv5_1:wgrad conv4_2:fwd conv4_2:dgrad conv1_2:fwdpool conv1_2:dgrad \
  --opts 'nt_halo=1,halo_wide=1,halo_min_splits=1,res64_pp=1' --opts 'nt_halo=0,halo_wide=1,halo_min_splits=1,res64_pp=1' \
  --opts 'nt_halo=1,halo_wide=0,halo_min_splits=1,res64_pp=1' --opts 'nt_halo=1,halo_wide=1,halo_min_splits=4,res64_pp=1' \
  --opts 'nt_halo=1,halo_wide=0,halo_min_splits=4,res64_pp=1' --opts 'nt_halo=1,halo_wide=1,halo_min_splits=1,res64_pp=0' --rounds 5 --reps 10 > $OUT/kbench_c5.txt 2>&1 || { tail -20 $OUT/kbench_c5.txt; exit 1; }
cat $OUT/kbench_c5.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_res64pp.py tests/test_gpu_pool_fusion.py tests/test_gpu_fcdensenet.py tests/test_gpu_dp_rccl.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_small.log 2>&1 || { tail -40 $OUT/pytest_small.log; exit 1; }
tail -2 $OUT/pytest_small.log
bash tools/ab_bench.sh r04_j2/ab "" "--schedule shadow_update=1" || exit 1
P="--steps 10 --warmup 3 --no-cpu-baseline --no-traffic --no-miou --no-pipeline --no-extra --no-inference --no-dp-probe"
timeout -k 10 300 python bench.py $P --model fcdensenet > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -30 $OUT/bench_c3.err; exit 1; }
cat $OUT/bench_c3.json
echo done
