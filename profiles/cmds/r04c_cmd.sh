#!/bin/bash
# round 4 (c): drop-in gap trace + publish-position A/B; decode parity + bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_decode.py tests/test_gpu_early.py \
  tests/test_gpu_dropin_memory.py -m gpu > gpurun_out/r04c_tests.log 2>&1 || exit $?
timeout -k 10 300 python tools/decode_bench.py > gpurun_out/r04c_decode_bench.txt 2>&1 || exit $?
bash tools/dropin_gaps.sh > gpurun_out/r04c_dropin_gaps.txt 2>&1 || exit $?
RTKV_K2_PUBLISH_LATE=1 DROPIN_OUT=late bash tools/dropin_gaps.sh > gpurun_out/r04c_dropin_gaps_late.txt 2>&1 || exit $?
