#!/bin/bash
# round 4 (k): drop-in prefetch size sweep (bench leg, 10 steps each)
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
for mb in 0 24 40 64; do
  RTKV_DROPIN_PREFETCH_MB=$mb $T 300 python bench.py --legs drop_in --steps 5 --warmup 2 --leg-steps 10 > gpurun_out/r04k_pf$mb.json 2> gpurun_out/r04k_pf$mb.err || exit $?
done
