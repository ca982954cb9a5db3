# decode shape sweep (RTKV_DECODE_SHAPE) under rocprof kernel stats
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp
for w in "$@"; do
  RTKV_DECODE_SHAPE=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/ps_$w -o dec -- python3 $GRAFT_REPO_ROOT/tools/decode_bench.py > $GRAFT_REPO_ROOT/gpurun_out/decps_$w.log 2>&1 || exit 1
done
