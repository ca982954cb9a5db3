#!/bin/bash
# round 4 (b): K1 split-head fp16/bf16 kernel + S-dependent K1 workgroup size; one-workgroup K2 for
# S <= 8192; mask kernel; parity + A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_select_fast.py tests/test_gpu_early.py tests/test_gpu_dropin_memory.py tests/test_gpu_stats.py tests/test_gpu_parity.py tests/test_gpu_shard.py \
  tests/test_gpu_model_side.py tests/test_gpu_model_side_ref.py tests/test_gpu_f32_masks.py tests/test_gpu_lse.py \
  -m gpu > gpurun_out/r04b_tests.log 2>&1 || exit $?
B="python bench.py --steps 10 --warmup 3 --legs none --cpu-baseline-seconds 0"
timeout -k 10 300 $B --dtype float16 > gpurun_out/r04b_f16_split.json 2>/dev/null || exit $?
RTKV_K1_NOSPLIT=1 timeout -k 10 300 $B --dtype float16 > gpurun_out/r04b_f16_nosplit.json 2>/dev/null || exit $?
timeout -k 10 300 $B --dtype bfloat16 > gpurun_out/r04b_bf16_split.json 2>/dev/null || exit $?
for dt in float32 float16; do
  timeout -k 10 300 $B --seq 4096 --dtype $dt > gpurun_out/r04b_s4096_${dt}_new.json 2>/dev/null || exit $?
  RTKV_K1_BT=1024 RTKV_K1_BT16=1024 RTKV_K1_NOSPLIT=1 RTKV_K2_ONE_MAXS=0 timeout -k 10 300 $B --seq 4096 --dtype $dt \
    > gpurun_out/r04b_s4096_${dt}_old.json 2>/dev/null || exit $?
  RTKV_K1_BT=256 timeout -k 10 300 $B --seq 4096 --dtype $dt > gpurun_out/r04b_s4096_${dt}_bt256.json 2>/dev/null || exit $?
  timeout -k 10 300 $B --seq 8192 --dtype $dt > gpurun_out/r04b_s8192_${dt}_one.json 2>/dev/null || exit $?
  RTKV_K2_ONE_MAXS=0 timeout -k 10 300 $B --seq 8192 --dtype $dt > gpurun_out/r04b_s8192_${dt}_multi.json 2>/dev/null || exit $?
done
RTKV_K2_ONE_MAXS=32768 timeout -k 10 300 $B > gpurun_out/r04b_f32_one16k.json 2>/dev/null || exit $?
RTKV_K2_ONE_MAXS=32768 timeout -k 10 300 $B --dtype float16 > gpurun_out/r04b_f16_one16k.json 2>/dev/null || exit $?
RTKV_K2_ONE_MAXS=32768 timeout -k 10 300 $B --seq 32768 --layers 8 > gpurun_out/r04b_s32k_one.json 2>/dev/null || exit $?
timeout -k 10 300 $B --seq 32768 --layers 8 > gpurun_out/r04b_s32k_multi.json 2>/dev/null || exit $?
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --legs drop_in --cpu-baseline-seconds 0 > gpurun_out/r04b_dropin.json 2>/dev/null || exit $?
bash tools/dropin_gaps.sh > gpurun_out/r04b_dropin_gaps.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_decode.py -m gpu > gpurun_out/r04b_decode_tests.log 2>&1 || exit $?
timeout -k 10 300 python tools/decode_bench.py > gpurun_out/r04b_decode_bench.txt 2>&1 || exit $?
