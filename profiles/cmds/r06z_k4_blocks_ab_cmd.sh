#!/usr/bin/env bash
# K4 grid cap A/B (RTKV_K4_BLOCKS) on the f16 packed-only workload
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
O=gpurun_out/r06z; mkdir -p $O
for rep in 1 2; do
for B in 0 1024 2048 4096; do
  if [ $B -eq 0 ]; then unset RTKV_K4_BLOCKS; else export RTKV_K4_BLOCKS=$B; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --dtype float16 --no-dequant --legs none --cpu-baseline-seconds 0 > $O/b_$B.json 2> $O/b_$B.err || { echo "rc=$?"; tail -5 $O/b_$B.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_$B.json').read().strip().splitlines()[-1]); print('$rep $B', d['ms_per_step'], d['kernel_us_per_layer'])"
done
done
