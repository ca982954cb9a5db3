#!/bin/bash
# round 4: the full GPU suite (incl. cfg4 reference goldens, late-timeout / overflow tests), the
# multi-rank bench rehearsal (gloo, 2 ranks on the one GPU), the launcher's fail-fast, a short bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r04a_tests.log 2>&1 || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 --dist-backend gloo --layers 4 --steps 2 --warmup 1 \
  > gpurun_out/r04a_gloo2.json 2> gpurun_out/r04a_gloo2.err || exit $?
rc=0; timeout -k 10 120 python bench.py --gpus 2 > gpurun_out/r04a_failfast.out 2>&1 || rc=$?
echo "failfast rc=$rc" >> gpurun_out/r04a_failfast.out
[ "$rc" = 2 ] || exit 3
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --legs none > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err || exit $?
# K2 Infinity-Cache prefetch A/B (RTKV_K2_PREFETCH_MB), fp32 and fp16 cfg3
for mb in 0 40 80 120; do
  RTKV_K2_PREFETCH_MB=$mb timeout -k 10 300 python bench.py --steps 10 --warmup 3 --legs none --cpu-baseline-seconds 0 \
    > gpurun_out/r04a_pf${mb}_f32.json 2>/dev/null || exit $?
  RTKV_K2_PREFETCH_MB=$mb timeout -k 10 300 python bench.py --steps 10 --warmup 3 --legs none --cpu-baseline-seconds 0 \
    --dtype float16 > gpurun_out/r04a_pf${mb}_f16.json 2>/dev/null || exit $?
done
