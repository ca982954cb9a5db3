#!/bin/bash
# round 4 (z): K1' grid target 512 vs 1024 (fused importance mode, cfg3 f16), then the final-tree bench
# line with all legs and a rocprofv3 kernel-stats pass of the headline
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10 240"
for r in 1 2; do
  for w in 1024 512; do
    RTKV_QK_WGS=$w $T python bench.py --dtype float16 --importance qk --legs none --steps 10 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/r04z_qk_wgs${w}_$r.json 2>/dev/null || exit $?
  done
done
timeout -k 10 600 python bench.py > gpurun_out/r04z_bench.json 2> gpurun_out/r04z_bench.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04z_prof -o r04z -- python3 $GRAFT_REPO_ROOT/bench.py --legs none --steps 20 --warmup 3 --cpu-baseline-seconds 0 > $GRAFT_REPO_ROOT/gpurun_out/r04z_prof.log 2>&1 || exit $?
