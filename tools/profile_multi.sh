# Round-end profiles of several bench workloads in one GPU call: per workload a rocprofv3 kernel-stats
# pass and separate-pass PMC FETCH_SIZE / WRITE_SIZE, each into gpurun_out/<tag>/{prof,pmc,pmcw}
# (summarised by: python profiles/summarize.py <tag> gpurun_out/<tag> -- <args>).
# WORKLOADS: lines "tag|bench args" (default: the headline and the bench legs' workloads).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
W="${WORKLOADS:-main|
pub16|--params pub16
f16|--dtype float16
pk|--no-dequant
f16pk|--dtype float16 --no-dequant
s4096|--seq 4096
cfg2q|--seq 4096 --quant-only}"
cd /tmp && export TMPDIR=/tmp
while IFS='|' read -r tag a; do
  [ -z "$tag" ] && continue
  o=$R/gpurun_out/$tag
  mkdir -p $o
  echo "== $tag ($a) $(date +%T)"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python3 $R/bench.py --legs none --cpu-baseline-seconds 0 --streams 1 $a > $o/prof.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/pmc -o fetch -- python3 $R/bench.py --steps 2 --warmup 1 --legs none --cpu-baseline-seconds 0 --streams 1 $a > $o/pmc.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/pmcw -o write -- python3 $R/bench.py --steps 2 --warmup 1 --legs none --cpu-baseline-seconds 0 --streams 1 $a > $o/pmcw.log 2>&1
  rm -f $o/prof/*kernel_trace.csv
  tail -n 1 $o/prof.log
done <<< "$W"
