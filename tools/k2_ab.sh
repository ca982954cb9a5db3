# K2 change check: selection parity (fast vs pipeline vs oracle, fused, early), the probe timeline, bench.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_select_fast.py tests/test_gpu_parity.py tests/test_gpu_early.py tests/test_gpu_stats.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/k2_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/k2_tests.log; exit 1; }
tail -2 gpurun_out/k2_tests.log
timeout -k 10 120 ./tools/k2_probe 16384 0.6 > gpurun_out/k2probe.txt 2>&1 || exit 1
head -22 gpurun_out/k2probe.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --legs f16 --cpu-baseline-seconds 0 > gpurun_out/k2_main.json 2>gpurun_out/k2_main.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/k2_main.json'));print('main',d['ms_per_step'],d['kernel_us_per_layer'],'f16',d['legs']['f16']['ms_per_step'],d['legs']['f16']['kernel_us_per_layer'])"
