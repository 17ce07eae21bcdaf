#!/bin/bash
# usage: tools/pmc_kb.sh OUTDIR SPEC [kbench opts...] -- three rocprofv3 counter passes over tools/kbench.py SPEC
set -o pipefail
OUT=$1; SPEC=$2; shift 2
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM"
P3="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE TCC_EA0_RDREQ_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/p$i -o run -- python tools/kbench.py $SPEC --reps 3 --rounds 1 "$@" > /dev/null 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
python tools/pmc_kb_summary.py $OUT
