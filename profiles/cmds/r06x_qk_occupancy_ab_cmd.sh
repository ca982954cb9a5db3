#!/usr/bin/env bash
# K1' (qk_head32_kernel) occupancy A/B: default (2 waves/SIMD, 2 tiles ahead) vs 3 or 4 waves/SIMD with 1 tile ahead
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
O=gpurun_out/r06x; mkdir -p $O
P=realtime-kv-cache-compression_amd
for rep in 1 2; do
for v in "librtkv.so 512" "librtkv_wpe3.so 768" "librtkv_wpe3.so 1024" "librtkv_wpe4.so 1024"; do
  set -- $v
  RTKV_LIB=$P/$1 RTKV_QK32_WGS=$2 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --importance qk --dtype float16 --legs none --cpu-baseline-seconds 0 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { echo "rc=$?"; tail -5 $O/b_$1_$2.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_$1_$2.json').read().strip().splitlines()[-1]); print('$rep $1 $2', d['ms_per_step'], d['kernel_us_per_layer'])"
done
done
