#!/usr/bin/env bash
# gq pack rewrite: parity tests, the bench's gq leg (fp32 main line, fp16), kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06t
O=gpurun_out/r06t
timeout -k 10 400 python -u -m pytest tests/test_gpu_gq.py tests/test_gpu_dropin_memory.py -x -v -s -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gq.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_gq.log; exit 1; }
tail -3 $O/pytest_gq.log; grep "device span" $O/pytest_gq.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --legs gq --leg-steps 3 --cpu-baseline-seconds 0 > $O/bench_gq_f32.json 2> $O/bench_gq_f32.err || { echo "bench rc=$?"; tail -20 $O/bench_gq_f32.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_gq_f32.json').read().strip().splitlines()[-1]); print('f32', d['legs']['gq']['us_per_layer'], d['legs']['gq']['side_stream'])"
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --dtype float16 --legs gq --leg-steps 3 --cpu-baseline-seconds 0 > $O/bench_gq_f16.json 2> $O/bench_gq_f16.err || { echo "bench16 rc=$?"; tail -20 $O/bench_gq_f16.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_gq_f16.json').read().strip().splitlines()[-1]); print('f16', d['legs']['gq']['us_per_layer'], d['legs']['gq']['side_stream'])"
for D in float32 float16; do timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$D -o run -- python3 bench.py --steps 2 --warmup 1 --dtype $D --legs gq --leg-steps 2 --cpu-baseline-seconds 0 > $O/prof_$D.log 2>&1 || { echo "prof rc=$?"; tail -20 $O/prof_$D.log; exit 1; }; done
for D in float32 float16; do grep -h -E "gq_" $O/prof_$D/run_kernel_stats.csv | cut -c1-160; done
