#!/bin/bash
# round 4 (ad): split-row K4 as the fp32 default at every S — full GPU suite, then the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ad_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/r04ad_bench.json 2> gpurun_out/r04ad_bench.err || exit $?
