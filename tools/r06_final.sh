# Round-6 final-tree evidence: the whole GPU suite, smoke(), the default bench line, rocprofv3 kernel
# stats and separate FETCH_SIZE / WRITE_SIZE passes of the default workload (profiles/summarize.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06_final}
mkdir -p $O
cd $R
timeout -k 10 1700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --legs none --cpu-baseline-seconds 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $B --steps 5 --warmup 2 > $O/prof.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc -o fetch -- python3 $B --steps 2 --warmup 1 > $O/pmc.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw -o write -- python3 $B --steps 2 --warmup 1 > $O/pmcw.log 2>&1 || exit 1
