set -e
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --legs none --cpu-baseline-seconds 0 > gpurun_out/ab_stage.log 2>&1
grep -o '"kernel_us_per_layer": {[^}]*}' gpurun_out/ab_stage.log
grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_stage.log
MODES="deq:--no-packed both:" bash tools/k4_pmc_split.sh
