#!/bin/bash
# round 4 (e): drop-in after the event / host-path changes: tests, gap trace, bench leg
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_early.py \
  tests/test_gpu_dropin_memory.py tests/test_gpu_stats.py -m gpu > gpurun_out/r04e_tests.log 2>&1 || exit $?
DROPIN_OUT=r04e bash tools/dropin_gaps.sh > gpurun_out/r04e_dropin_gaps.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --legs drop_in --steps 10 --warmup 3 --leg-steps 10 > gpurun_out/r04e_bench.json 2> gpurun_out/r04e_bench.err || exit $?
for mb in 32 64 96; do
  RTKV_DROPIN_PREFETCH_MB=$mb DROPIN_OUT=r04e_pf$mb bash tools/dropin_gaps.sh > gpurun_out/r04e_dropin_gaps_pf$mb.txt 2>&1 || exit $?
done
RTKV_DROPIN_PREFETCH_MB=64 timeout -k 10 300 python bench.py --legs drop_in --steps 10 --warmup 3 --leg-steps 10 > gpurun_out/r04e_bench_pf64.json 2> gpurun_out/r04e_bench_pf64.err || exit $?
