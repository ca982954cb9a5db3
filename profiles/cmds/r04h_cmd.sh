#!/bin/bash
# round 4 (h): pooled processing_time events — drop-in tests, gap trace, drop-in leg
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dropin_memory.py tests/test_gpu_early.py \
  tests/test_gpu_stats.py -m gpu > gpurun_out/r04h_tests.log 2>&1 || exit $?
DROPIN_OUT=r04h bash tools/dropin_gaps.sh > gpurun_out/r04h_dropin_gaps.txt 2>&1 || exit $?
$T 300 python bench.py --legs drop_in --steps 5 --warmup 2 --leg-steps 10 > gpurun_out/r04h_dropin.json 2> gpurun_out/r04h_dropin.err || exit $?
