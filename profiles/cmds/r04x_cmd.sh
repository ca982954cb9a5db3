#!/bin/bash
# round 4 (x): drop-in outputs from a private allocator pool (RTKV_DROPIN_POOL=1) — memory test and the leg after others
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10 300"
RTKV_DROPIN_POOL=1 $T python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dropin_memory.py tests/test_gpu_early.py -m gpu > gpurun_out/r04x_tests.log 2>&1 || exit $?
for v in 0 1; do
  RTKV_DROPIN_POOL=$v $T python bench.py --legs f16,packed_only,drop_in --steps 5 --warmup 2 --leg-steps 10 --cpu-baseline-seconds 0 > gpurun_out/r04x_after_pool$v.json 2>/dev/null || exit $?
  RTKV_DROPIN_POOL=$v $T python bench.py --legs drop_in --steps 5 --warmup 2 --leg-steps 10 --cpu-baseline-seconds 0 > gpurun_out/r04x_alone_pool$v.json 2>/dev/null || exit $?
done
