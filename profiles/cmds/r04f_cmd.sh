#!/bin/bash
# round 4 (f): split-row K4 (short layers) parity + A/B; drop-in after the host-path changes (+ prefetch A/B)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k split_row_k4 \
  tests/test_gpu_early.py tests/test_gpu_dropin_memory.py tests/test_gpu_stats.py tests/test_gpu_decode.py -m gpu > gpurun_out/r04f_tests.log 2>&1 || exit $?
$T 300 python tools/decode_bench.py > gpurun_out/r04f_decode_bench.txt 2>&1 || exit $?
for v in 8192 0; do
  RTKV_K4_SPLIT_MAXS=$v $T 300 python bench.py --legs s4096,cfg2_s4096_quant --steps 5 --warmup 2 --leg-steps 10 > gpurun_out/r04f_s4096_split$v.json 2> gpurun_out/r04f_s4096_split$v.err || exit $?
  RTKV_K4_SPLIT_MAXS=$v $T 300 python bench.py --seq 8192 --layers 16 --legs none --steps 10 --warmup 3 > gpurun_out/r04f_s8192_split$v.json 2> gpurun_out/r04f_s8192_split$v.err || exit $?
  RTKV_K4_SPLIT_MAXS=$v $T 300 python bench.py --seq 8192 --layers 16 --dtype float16 --legs none --steps 10 --warmup 3 > gpurun_out/r04f_s8192f16_split$v.json 2> gpurun_out/r04f_s8192f16_split$v.err || exit $?
done
DROPIN_OUT=r04f bash tools/dropin_gaps.sh > gpurun_out/r04f_dropin_gaps.txt 2>&1 || exit $?
RTKV_DROPIN_PREFETCH_MB=64 DROPIN_OUT=r04f_pf64 bash tools/dropin_gaps.sh > gpurun_out/r04f_dropin_gaps_pf64.txt 2>&1 || exit $?
for mb in 0 64; do
  RTKV_DROPIN_PREFETCH_MB=$mb $T 300 python bench.py --legs drop_in --steps 5 --warmup 2 --leg-steps 10 > gpurun_out/r04f_dropin_pf$mb.json 2> gpurun_out/r04f_dropin_pf$mb.err || exit $?
done
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_qk.py -m gpu > gpurun_out/r04f_qk_tests.log 2>&1 || exit $?
for ah in 1 2; do
  RTKV_QK_AHEAD=$ah $T 300 python bench.py --importance qk --dtype float16 --legs none --steps 10 --warmup 3 > gpurun_out/r04f_qk_ahead$ah.json 2> gpurun_out/r04f_qk_ahead$ah.err || exit $?
done
