# K4 HBM traffic by output mode: FETCH_SIZE and WRITE_SIZE (separate rocprofv3 passes) of the fp32
# headline workload with both outputs, packed codes only, and dequantized rows only
# (DTYPE=float16 for the fp16 workload; MODES="deq:--no-packed" for one mode).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/k4split
cd /tmp && export TMPDIR=/tmp
DT=${DTYPE:-float32}
for V in ${MODES:-both:"" packed:"--no-dequant" deq:"--no-packed"}; do
  tag=${V%%:*}_$DT; flags=${V#*:}
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/k4split -o ${tag}_$C -- python3 $R/bench.py --steps 2 --warmup 1 --legs none --cpu-baseline-seconds 0 --layers 8 --dtype $DT $flags > $R/gpurun_out/k4split/${tag}_$C.log 2>&1
  done
done
