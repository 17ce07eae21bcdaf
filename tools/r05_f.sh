#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r05_f}; mkdir -p $OUT; export TMPDIR=/tmp
for s in conv6:wgrad conv6:wgrad_adam conv3_2:wgrad conv4_2:fwd conv7:wgrad; do
  echo "### $s"; bash tools/pmc_kb.sh $OUT/$(echo $s | tr ':' '_') $s || exit 1
done
