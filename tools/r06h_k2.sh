# K2 check: the selection tests, the K2 probe (partly kept and all-kept layers), the default bench line.
set -o pipefail
O=gpurun_out/${TAG:-r06i}
mkdir -p $O
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 900 python -u -m pytest tests/test_gpu_select_fast.py tests/test_gpu_early.py tests/test_gpu_parity.py tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for a in "16384 0.6" "16384 1.0" "4096 0.6" "4096 1.0" "65536 0.6"; do
  timeout -k 10 120 ./tools/k2_probe $a > $O/k2probe_$(echo $a | tr ' ' _).txt 2>&1 || exit 1
done
[ -n "${SKIP_BENCH:-}" ] || timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
