#!/bin/bash
# round 4 (ab): split-row K4 at cfg3 (S = 16384 fp32; RTKV_K4_SPLIT_MAXS=16384) against the whole-row
# kernel (default bound 8192), interleaved on one box
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10 240"
for r in 1 2; do
  $T python bench.py --legs none --steps 10 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/r04ab_whole_$r.json 2>/dev/null || exit $?
  RTKV_K4_SPLIT_MAXS=16384 $T python bench.py --legs none --steps 10 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/r04ab_split_$r.json 2>/dev/null || exit $?
done
