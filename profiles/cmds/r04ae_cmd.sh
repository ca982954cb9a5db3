#!/bin/bash
# round 4 (ae): final tree with the split-row K4 default for fp32 — kernel stats, FETCH_SIZE and
# WRITE_SIZE passes (each its own run) of the headline, then the default bench line
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
B="$R/bench.py --steps 2 --warmup 1 --legs none --cpu-baseline-seconds 0"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --legs none --steps 20 --warmup 3 --cpu-baseline-seconds 0 > $R/gpurun_out/r04ae_prof.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc -o fetch --output-format csv -- python3 $B > $R/gpurun_out/r04ae_pmc.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmcw -o write --output-format csv -- python3 $B > $R/gpurun_out/r04ae_pmcw.log 2>&1 || exit $?
cd $R
timeout -k 10 600 python bench.py > gpurun_out/r04ae_bench.json 2> gpurun_out/r04ae_bench.err || exit $?
