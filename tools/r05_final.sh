#!/bin/bash
# end of round: full GPU suite + smoke, then the measurement set (tools/r05_measure.sh)
set -o pipefail
TAG=${1:-r05_final}
bash tools/r05_tests.sh ${TAG}_t && bash tools/r05_measure.sh ${TAG}_m
