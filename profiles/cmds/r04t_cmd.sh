#!/bin/bash
# round 4 (t): fp32 K1 at 512 threads (short layers): 4 / 8 / 16 heads per load batch — parity and s4096 A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for hb in 8 16; do
  RTKV_K1_HB32=$hb timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "register_aggregation or aggregation_scores or compress_layer_kv_cache" -m gpu > gpurun_out/r04t_tests_hb$hb.log 2>&1 || exit $?
done
for hb in 0 8 16; do
  RTKV_K1_HB32=$hb timeout -k 10 300 python bench.py --legs s4096,cfg2_s4096_quant --steps 5 --warmup 2 --leg-steps 10 --cpu-baseline-seconds 0 > gpurun_out/r04t_hb$hb.json 2>/dev/null || exit $?
done
