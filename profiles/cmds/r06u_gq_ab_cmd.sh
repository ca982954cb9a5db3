#!/usr/bin/env bash
# gq pack grid A/B (RTKV_GQ_PACK_WGS) on the bench's gq leg, fp32 and fp16
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
O=gpurun_out/r06u; mkdir -p $O
for rep in 1 2; do
for W in 8192 1024 512 2048; do
  for D in float32 float16; do
    RTKV_GQ_PACK_WGS=$W timeout -k 10 300 python bench.py --steps 2 --warmup 1 --dtype $D --legs gq --leg-steps 3 --cpu-baseline-seconds 0 > $O/b_${W}_${D}.json 2> $O/b_${W}_${D}.err || { echo "rc=$?"; tail -5 $O/b_${W}_${D}.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${W}_${D}.json').read().strip().splitlines()[-1]); print('$rep $W $D', d['legs']['gq']['us_per_layer'])"
  done
done
done
