#!/usr/bin/env bash
# Kernel trace of the drop-in path (RealTimePrefillCompressor.compress_layer_kv_cache over the 32 cfg3
# layers): per-kernel durations and the idle gap before each kernel, i.e. how long the device waits for
# the host between K2's early publication and K4's launch (rocprofv3 --kernel-trace; no counters).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/dropin_gaps${DROPIN_OUT:+_$DROPIN_OUT}
rm -rf "$out"; mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$out" -o trace -- python3 tools/dropin_profile.py \
  --layers 32 --reps 5 --no-cprofile ${DROPIN_ARGS:-} > "$out/run.log" 2>&1
python3 tools/gap_summary.py "$out" --layers 32 --warmup 2 --reps 5 > "$out/summary.txt"
cat "$out/run.log" | grep -v amdgpu.ids; cat "$out/summary.txt"
