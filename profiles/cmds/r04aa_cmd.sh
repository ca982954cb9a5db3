#!/bin/bash
# round 4 (aa): K1' head kernel without the key-bias adds when there is no key bias (bit-identical),
# parity tests, then interleaved A/B against the previous form (librtkv_qkold.so, -DRTKV_QK_OLD)
set -o pipefail
mkdir -p gpurun_out
L=realtime-kv-cache-compression_amd
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_qk.py -m gpu > gpurun_out/r04aa_tests.log 2>&1 || exit $?
T="timeout -k 10 240"
for r in 1 2; do
  $T python bench.py --dtype float16 --importance qk --legs none --steps 10 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/r04aa_new_$r.json 2>/dev/null || exit $?
  RTKV_LIB=$L/librtkv_qkold.so $T python bench.py --dtype float16 --importance qk --legs none --steps 10 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/r04aa_old_$r.json 2>/dev/null || exit $?
done
