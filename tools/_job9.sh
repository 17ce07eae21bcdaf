set -o pipefail
OUT=gpurun_out/r04_j9; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_bench.sh r04_j9/ab "" "--option adam_tr_fused=1" "--schedule fused_delay=4" "--schedule fused_delay=9" "--schedule main_wgrad=0" "--option tn_fill=3" || exit 1
echo done
