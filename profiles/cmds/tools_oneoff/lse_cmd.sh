set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_lse.py tests/test_gpu_f32_masks.py tests/test_gpu_model_side.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/lse_tests.log 2>&1 || { tail -30 gpurun_out/lse_tests.log; exit 1; }
tail -2 gpurun_out/lse_tests.log
for k in 16 32; do RTKV_LSE_KERNEL=$k timeout -k 10 120 python tools/lse_bench.py 16384 32 float16; done
timeout -k 10 120 python tools/lse_bench.py 16384 32 float16 64
for k in 16 32; do RTKV_LSE_KERNEL=$k timeout -k 10 120 python tools/lse_bench.py 16384 32 bfloat16; done
timeout -k 10 120 python tools/lse_bench.py 16384 32 float32
