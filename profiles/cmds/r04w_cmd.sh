#!/bin/bash
# round 4 (w): drop-in leg alone and after the f16 / packed-only legs, with the raw driver re-measured
# in the same state right before it
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10 300"
$T python bench.py --legs drop_in --steps 5 --warmup 2 --leg-steps 10 --cpu-baseline-seconds 0 > gpurun_out/r04w_alone.json 2>/dev/null || exit $?
$T python bench.py --legs f16,packed_only,drop_in --steps 5 --warmup 2 --leg-steps 10 --cpu-baseline-seconds 0 > gpurun_out/r04w_after.json 2>/dev/null || exit $?
