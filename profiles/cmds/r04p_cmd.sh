#!/bin/bash
# round 4 (p): new early/drop-in tests; bench line picks up profiles/r04_pmc.json
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_early.py tests/test_gpu_dropin_memory.py -m gpu > gpurun_out/r04p_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --legs none --steps 10 --warmup 3 > gpurun_out/r04p_bench.json 2> gpurun_out/r04p_bench.err || exit $?
timeout -k 10 300 python tools/dropin_profile.py --layers 32 --reps 5 --stamps > gpurun_out/r04p_stamps.txt 2>&1 || exit $?
RTKV_DROPIN_PREFETCH_MB=0 timeout -k 10 300 python tools/dropin_profile.py --layers 32 --reps 5 --stamps > gpurun_out/r04p_stamps_pf0.txt 2>&1 || exit $?
for w in 1024 2048 4096; do
  RTKV_QK_WGS=$w timeout -k 10 300 python bench.py --importance qk --dtype float16 --legs none --steps 5 --warmup 2 --cpu-baseline-seconds 0 > gpurun_out/r04p_qk_wgs$w.json 2>/dev/null || exit $?
done
RTKV_K1_HB16=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "compress_layer_kv_cache and cfg3 or aggregation" -m gpu > gpurun_out/r04p_k1hb_tests.log 2>&1 || exit $?
for hb in 0 8 4; do
  RTKV_K1_HB16=$hb timeout -k 10 300 python bench.py --dtype float16 --legs none --steps 10 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/r04p_k1hb$hb.json 2>/dev/null || exit $?
done
RTKV_QK_NWV=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_qk.py -m gpu > gpurun_out/r04p_qk8_tests.log 2>&1 || exit $?
for nw in 4 8; do
  RTKV_QK_NWV=$nw timeout -k 10 300 python bench.py --importance qk --dtype float16 --legs none --steps 5 --warmup 2 --cpu-baseline-seconds 0 > gpurun_out/r04p_qk_nwv$nw.json 2>/dev/null || exit $?
done
