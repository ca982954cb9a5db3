#!/usr/bin/env bash
# Kernel trace of the sequential bench step: per-kernel durations and the idle gaps between
# consecutive kernels (rocprofv3 --kernel-trace; no counters).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/gaps
rm -rf "$out"; mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$out" -o trace -- python3 bench.py --steps 3 --warmup 1 --legs none --cpu-baseline-seconds 0 ${BENCH_ARGS:-} > "$out/bench.log" 2>&1
python3 tools/gap_summary.py "$out" > "$out/summary.txt"
cat "$out/summary.txt"
