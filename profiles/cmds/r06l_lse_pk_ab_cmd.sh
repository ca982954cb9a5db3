#!/usr/bin/env bash
# LSE kernel with packed-fp32 fma/add: bit-identity against the previous build, interleaved timing A/B, tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
O=gpurun_out/r06l; mkdir -p $O
P=realtime-kv-cache-compression_amd
RTKV_LIB=$P/librtkv_old.so timeout -k 10 200 python tools/lse_bitcmp.py save $O/old.pt > $O/bit.log 2>&1 || { echo "save old failed"; tail $O/bit.log; exit 1; }
timeout -k 10 200 python tools/lse_bitcmp.py save $O/new.pt >> $O/bit.log 2>&1 || { echo "save new failed"; tail $O/bit.log; exit 1; }
timeout -k 10 100 python tools/lse_bitcmp.py cmp $O/old.pt $O/new.pt > $O/bitcmp.log 2>&1; rc=$?; cat $O/bitcmp.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  for L in librtkv_old.so librtkv.so; do
    for D in float16 bfloat16; do
      RTKV_LIB=$P/$L timeout -k 10 200 python tools/lse_bench.py 16384 32 $D 2>&1 | tail -1 | sed "s/^/$rep $L /"
    done
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_lse.py tests/test_gpu_qk.py tests/test_gpu_fused_mismatch.py tests/test_gpu_model_side.py tests/test_gpu_model_side_ref.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED" $O/pytest.log | head; exit 1; }
