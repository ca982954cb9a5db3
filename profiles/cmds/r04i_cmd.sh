#!/bin/bash
# round 4 (i): what costs the drop-in's extra ~5 us before K1: start event / timing events A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
RTKV_AB_NOSTART=1 DROPIN_OUT=r04i_nostart bash tools/dropin_gaps.sh > gpurun_out/r04i_nostart.txt 2>&1 || exit $?
RTKV_AB_NOSTART=1 RTKV_AB_NOTIMING=1 DROPIN_OUT=r04i_nostart_notiming bash tools/dropin_gaps.sh > gpurun_out/r04i_nn.txt 2>&1 || exit $?
RTKV_DROPIN_PREFETCH_MB=0 RTKV_AB_NOSTART=1 RTKV_AB_NOTIMING=1 DROPIN_OUT=r04i_nn_pf0 bash tools/dropin_gaps.sh > gpurun_out/r04i_nn_pf0.txt 2>&1 || exit $?
