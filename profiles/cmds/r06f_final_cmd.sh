#!/usr/bin/env bash
# final-tree evidence: GPU suite, smoke, default bench line, kernel stats of the default workload
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
O=gpurun_out/r06f; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print({k: d[k] for k in ('value','ms_per_step')}, d['roofline']['frac'], d['kernel_us_per_layer'], d['legs']['gq']['us_per_layer'], d['legs']['prefill_7b'].get('fused_overhead_ms'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 1 --legs none --cpu-baseline-seconds 0 > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -5 $O/prof.log; exit 1; }
head -5 $O/prof/run_kernel_stats.csv | cut -c1-150
