#!/bin/bash
# round 4 (y): fp16 K1 with plain (cached) loads against non-temporal loads, cfg3 fp16, interleaved A/B
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10 240"
L=realtime-kv-cache-compression_amd
for r in 1 2; do
  $T python bench.py --dtype float16 --legs none --steps 10 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/r04y_nt_$r.json 2>/dev/null || exit $?
  RTKV_LIB=$L/librtkv_k1plain.so $T python bench.py --dtype float16 --legs none --steps 10 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/r04y_plain_$r.json 2>/dev/null || exit $?
done
