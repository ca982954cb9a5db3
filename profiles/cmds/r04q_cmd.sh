#!/bin/bash
# round 4 (q): K1' grid default 1024 — fused-mode tests and bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_qk.py tests/test_gpu_model_side.py tests/test_gpu_model_side_ref.py tests/test_gpu_f32_masks.py tests/test_gpu_shard.py -m gpu > gpurun_out/r04q_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --importance qk --dtype float16 --legs none --steps 10 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/r04q_qk.json 2>/dev/null || exit $?
