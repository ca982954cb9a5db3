#!/bin/bash
# round 4 (d): drop-in host overhead — cProfile + kernel-trace gaps after lazy views / deferred events
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_early.py \
  tests/test_gpu_dropin_memory.py tests/test_gpu_stats.py tests/test_gpu_parity.py -m gpu > gpurun_out/r04d_tests.log 2>&1 || exit $?
timeout -k 10 300 python tools/dropin_profile.py --layers 32 --reps 5 > gpurun_out/r04d_cprofile.txt 2>&1 || exit $?
DROPIN_OUT=r04d bash tools/dropin_gaps.sh > gpurun_out/r04d_dropin_gaps.txt 2>&1 || exit $?
RTKV_DROPIN_EVENTS=0 DROPIN_OUT=r04d_noev bash tools/dropin_gaps.sh > gpurun_out/r04d_dropin_gaps_noev.txt 2>&1 || exit $?
