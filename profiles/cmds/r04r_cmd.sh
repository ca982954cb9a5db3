#!/bin/bash
# round 4 (r): final tree — full GPU suite, smoke, the multi-rank bench rehearsal (gloo, 2 ranks on the
# one GPU), the launcher's fail-fast, a default-config bench line (no extra legs)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04r_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04r_smoke.log 2>&1 || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29631 bench.py --gpus 2 --dist-backend gloo --layers 4 --steps 2 --warmup 1 \
  > gpurun_out/r04r_gloo2.json 2> gpurun_out/r04r_gloo2.err || exit $?
rc=0; timeout -k 10 120 python bench.py --gpus 2 > gpurun_out/r04r_failfast.out 2>&1 || rc=$?
echo "failfast rc=$rc" >> gpurun_out/r04r_failfast.out
[ "$rc" = 2 ] || exit 3
