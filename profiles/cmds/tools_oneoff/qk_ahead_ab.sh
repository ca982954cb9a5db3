# A/B of K1' query prefetch depth (RTKV_QK_AHEAD) + the K2 early-load change; parity first.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_qk.py tests/test_gpu_select_fast.py tests/test_gpu_parity.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --legs f16 --cpu-baseline-seconds 0 > gpurun_out/ab_main.json 2>gpurun_out/ab_main.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/ab_main.json'));print('main',d['ms_per_step'],d['kernel_us_per_layer'],'f16',d['legs']['f16']['kernel_us_per_layer'])"
for a in 1 2 1 2; do
  RTKV_QK_AHEAD=$a timeout -k 10 300 python bench.py --importance qk --dtype float16 --steps 5 --warmup 2 --legs none --cpu-baseline-seconds 0 > gpurun_out/qk_ahead$a.json 2>gpurun_out/qk_ahead$a.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/qk_ahead$a.json'));print('ahead',$a,d['kernel_us_per_layer'],d['k1_mfma'])"
done
