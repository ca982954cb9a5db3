# decode: tests, then rocprof kernel stats of tools/decode_bench.py at several workgroup targets
mkdir -p gpurun_out && timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode.py > gpurun_out/dec.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for w in "$@"; do
  RTKV_DECODE_WGS=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/pd_$w -o dec -- python3 $GRAFT_REPO_ROOT/tools/decode_bench.py > $GRAFT_REPO_ROOT/gpurun_out/decprof_$w.log 2>&1 || exit 1
done
