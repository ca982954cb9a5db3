set -e
bash tools/lse_cmd.sh
bash tools/mfma_pmc.sh
timeout -k 10 300 python bench.py --legs none --cpu-baseline-seconds 0 > gpurun_out/ab_default.log 2>&1
timeout -k 10 300 python bench.py --legs none --cpu-baseline-seconds 0 --fused-quant > gpurun_out/ab_fused.log 2>&1
grep -o '"kernel_us_per_layer": {[^}]*}' gpurun_out/ab_default.log gpurun_out/ab_fused.log
grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_default.log gpurun_out/ab_fused.log
bash tools/k4_pmc_split.sh
