#!/bin/bash
# round 4 (u): rocprofv3 kernel stats + FETCH/WRITE passes for the S = 4096 and the f16 cfg3 workloads
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for tag in s4096 f16; do
  if [ $tag = s4096 ]; then A="--seq 4096"; else A="--dtype float16"; fi
  D=$R/gpurun_out/u_$tag
  mkdir -p $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 $R/bench.py --legs none --cpu-baseline-seconds 0 $A > $D/bench_prof.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pmc -o fetch -- python3 $R/bench.py --steps 2 --warmup 1 --legs none --cpu-baseline-seconds 0 $A > $D/pmc.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/pmcw -o write -- python3 $R/bench.py --steps 2 --warmup 1 --legs none --cpu-baseline-seconds 0 $A > $D/pmcw.log 2>&1
done
