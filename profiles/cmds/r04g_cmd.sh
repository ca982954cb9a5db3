#!/bin/bash
# round 4 (g): full GPU suite; drop-in host timeline; fp16 split-K4 A/B at S = 4096; drop-in leg (prefetch on)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r04g_pytest_gpu.log 2>&1 || exit $?
$T 300 python tools/dropin_profile.py --layers 32 --reps 5 --host-timeline > gpurun_out/r04g_host_timeline.txt 2>&1 || exit $?
for v in 4096 0; do
  RTKV_K4_SPLIT_MAXS=$v $T 300 python bench.py --dtype float16 --legs s4096 --steps 5 --warmup 2 --leg-steps 10 > gpurun_out/r04g_f16_s4096_split$v.json 2> gpurun_out/r04g_f16_s4096_split$v.err || exit $?
done
$T 300 python bench.py --legs drop_in --steps 5 --warmup 2 --leg-steps 10 > gpurun_out/r04g_dropin.json 2> gpurun_out/r04g_dropin.err || exit $?
