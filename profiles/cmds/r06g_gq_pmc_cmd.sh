#!/usr/bin/env bash
# FETCH_SIZE / WRITE_SIZE of the gq leg's kernels (separate counter passes) + kernel stats, fp32 and fp16
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
O=gpurun_out/r06g; mkdir -p $O
for D in float32 float16; do
  A="bench.py --steps 1 --warmup 1 --dtype $D --legs gq --leg-steps 2 --cpu-baseline-seconds 0"
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$D -o fetch -- python3 $A > $O/pmc_$D.log 2>&1 || { echo "fetch rc=$?"; tail -5 $O/pmc_$D.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw_$D -o write -- python3 $A > $O/pmcw_$D.log 2>&1 || { echo "write rc=$?"; tail -5 $O/pmcw_$D.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$D -o run -- python3 $A > $O/prof_$D.log 2>&1 || { echo "prof rc=$?"; tail -5 $O/prof_$D.log; exit 1; }
  grep -h "gq_" $O/prof_$D/run_kernel_stats.csv | cut -c1-150
done
