#!/bin/bash
# round 4 (ac): split-row K4 bound — fp16 cfg3 (S = 16384) and the fp32 S = 65536 leg, split vs whole row
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10 300"
for r in 1 2; do
  $T python bench.py --dtype float16 --legs none --steps 10 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/r04ac_f16_whole_$r.json 2>/dev/null || exit $?
  RTKV_K4_SPLIT_MAXS=16384 $T python bench.py --dtype float16 --legs none --steps 10 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/r04ac_f16_split_$r.json 2>/dev/null || exit $?
done
$T python bench.py --legs s65536 --steps 3 --warmup 1 --leg-steps 5 --cpu-baseline-seconds 0 > gpurun_out/r04ac_s65536_whole.json 2>/dev/null || exit $?
RTKV_K4_SPLIT_MAXS=65536 $T python bench.py --legs s65536 --steps 3 --warmup 1 --leg-steps 5 --cpu-baseline-seconds 0 > gpurun_out/r04ac_s65536_split.json 2>/dev/null || exit $?
