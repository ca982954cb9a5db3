#!/bin/bash
# round 4 (j): processing_time from kernel stamps (no events around the layer): tests, gap trace, legs
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dropin_memory.py tests/test_gpu_early.py \
  tests/test_gpu_stats.py tests/test_gpu_model_side.py tests/test_gpu_qk.py -m gpu > gpurun_out/r04j_tests.log 2>&1 || exit $?
DROPIN_OUT=r04j bash tools/dropin_gaps.sh > gpurun_out/r04j_dropin_gaps.txt 2>&1 || exit $?
$T 300 python bench.py --legs drop_in --steps 10 --warmup 3 --leg-steps 10 > gpurun_out/r04j_bench.json 2> gpurun_out/r04j_bench.err || exit $?
