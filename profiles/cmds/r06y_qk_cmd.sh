#!/usr/bin/env bash
# K1' at four waves per SIMD: qk / model-side / LSE tests, fused-mode bench line, kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
O=gpurun_out/r06y; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_qk.py tests/test_gpu_model_side_ref.py tests/test_gpu_fused_mismatch.py tests/test_gpu_model_side.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_qk.log 2>&1; rc=$?
tail -3 $O/pytest_qk.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_qk.log | head; exit 1; }
for rep in 1 2; do
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --importance qk --dtype float16 --legs none --cpu-baseline-seconds 0 > $O/b_qk.json 2> $O/b_qk.err || { echo "rc=$?"; tail -5 $O/b_qk.err; exit 1; }
python -c "import json; d=json.loads(open('$O/b_qk.json').read().strip().splitlines()[-1]); print('qk f16', d['ms_per_step'], d['kernel_us_per_layer'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 --importance qk --dtype float16 --legs none --cpu-baseline-seconds 0 > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -5 $O/prof.log; exit 1; }
grep -h -E "qk_head" $O/prof/run_kernel_stats.csv | cut -c1-160
SKIP_LSE=1 timeout -k 10 600 bash tools/mfma_pmc.sh > $O/mfma.log 2>&1 || { echo "mfma rc=$?"; tail -5 $O/mfma.log; exit 1; }
python tools/mfma_summary.py r06y gpurun_out/mfma > $O/mfma_summary.log 2>&1; tail -5 $O/mfma_summary.log; ls profiles/r06y_mfma.json && cp profiles/r06y_mfma.json $O/
