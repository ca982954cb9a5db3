#!/bin/bash
# round 4 (o): the round-end bench line (all legs), rocprofv3 kernel stats + FETCH/WRITE passes, MFMA counters
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash tools/profile_bench.sh || exit $?
bash tools/mfma_pmc.sh || exit $?
