#!/bin/bash
# round 4 (af): split-row K4 with head-strided outputs (the drop-in's exact-size K'/V') — full GPU
# suite, then the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04af_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/r04af_bench.json 2> gpurun_out/r04af_bench.err || exit $?
