#!/bin/bash
# round 4 (m): 8-wave split-row K4 A/B at S = 4096 / 8192 (fp32), parity of the 8-wave variant
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="timeout -k 10"
RTKV_K4_SPLIT8=1 $T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "split_row" -m gpu > gpurun_out/r04m_tests.log 2>&1 || exit $?
for v in 0 1; do
  RTKV_K4_SPLIT8=$v $T 300 python bench.py --legs s4096,cfg2_s4096_quant --steps 5 --warmup 2 --leg-steps 10 > gpurun_out/r04m_s4096_$v.json 2> gpurun_out/r04m_s4096_$v.err || exit $?
  RTKV_K4_SPLIT8=$v $T 300 python bench.py --seq 8192 --layers 16 --legs none --steps 10 --warmup 3 > gpurun_out/r04m_s8192_$v.json 2> gpurun_out/r04m_s8192_$v.err || exit $?
done
