# Round-end measurement: bench line, rocprofv3 kernel stats of the same workload, and separate-pass
# PMC FETCH_SIZE / WRITE_SIZE (summarised by: python profiles/summarize.py TAG gpurun_out -- $BENCH_ARGS).
# BENCH_ARGS selects the workload (default: bench.py's default, cfg3 fp32).  The profiled runs keep
# one layer stream, so each kernel's rocprof duration is its own (the bench line overlaps layers).
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
A="${BENCH_ARGS:-}"
timeout -k 10 500 python -u bench.py $A > gpurun_out/bench_line.json 2> gpurun_out/bench_err.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --legs none --cpu-baseline-seconds 0 --streams 1 $A > $R/gpurun_out/bench_prof.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc -o fetch -- python3 $R/bench.py --steps 2 --warmup 1 --legs none --cpu-baseline-seconds 0 --streams 1 $A > $R/gpurun_out/pmc.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcw -o write -- python3 $R/bench.py --steps 2 --warmup 1 --legs none --cpu-baseline-seconds 0 --streams 1 $A > $R/gpurun_out/pmcw.log 2>&1
