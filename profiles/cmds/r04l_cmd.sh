#!/bin/bash
# round 4 (l): K4 write-through (sc1) dequant stores A/B — K4 time and the K4 -> K1 gap
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="timeout -k 10"
V=$PWD/realtime-kv-cache-compression_amd/librtkv_sc1.so
RTKV_LIB=$V $T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "compress_layer or split_row or packed_only" -m gpu > gpurun_out/r04l_tests_sc1.log 2>&1 || exit $?
for v in base sc1; do
  if [ $v = sc1 ]; then export RTKV_LIB=$V; else unset RTKV_LIB; fi
  $T 300 python bench.py --legs none --steps 10 --warmup 3 > gpurun_out/r04l_$v.json 2> gpurun_out/r04l_$v.err || exit $?
  $T 300 python bench.py --legs none --dtype float16 --steps 10 --warmup 3 > gpurun_out/r04l_${v}_f16.json 2> gpurun_out/r04l_${v}_f16.err || exit $?
  DROPIN_OUT=r04l_$v bash tools/dropin_gaps.sh > gpurun_out/r04l_gaps_$v.txt 2>&1 || exit $?
done
