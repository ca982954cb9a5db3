set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_qk.py tests/test_gpu_model_side.py tests/test_gpu_model_side_ref.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/qk32_tests.log 2>&1 || { tail -30 gpurun_out/qk32_tests.log; exit 1; }
tail -3 gpurun_out/qk32_tests.log
timeout -k 10 600 python tools/ab_env.py qk32 --rounds 2 --variants 'k32=' 'k16=RTKV_QK16=1' -- --importance qk --dtype float16 --steps 10 --warmup 3 > gpurun_out/ab_qk32.log 2>&1
tail -4 gpurun_out/ab_qk32.log
