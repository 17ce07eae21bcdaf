#!/bin/bash
# usage: tools/pmc.sh OUTDIR LAYER OP VARIANT  -- three counter passes on one conv op
set -e
OUT=$1; L=$2; OP=$3; V=$4
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_UNALIGNED_STALL"
P3="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE TCC_EA0_RDREQ_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/${L}_${OP}_v${V}_p$i -o run -- python tools/one_conv.py $L $OP $V 5 > /dev/null 2>&1
done
