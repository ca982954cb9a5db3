#!/usr/bin/env bash
# GPU session script: every GPU step has its own time limit; stop at the first crash-like exit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in ${STEPS:-smoke pytest bench}; do
  case $s in
    smoke)  step smoke 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" ;;
    pytest) step pytest_gpu 1200 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    shardp) step shardp 900 python -u -m pytest tests/test_gpu_shard_procs.py tests/test_gpu_shard.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    early)  step early 600 python -u -m pytest tests/test_gpu_early.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    targ)   step targ 900 python -u -m pytest ${TESTS:-tests/test_gpu_f32_masks.py} -q -x -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    profprefill) step profprefill 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profprefill -o run -- python3 bench.py --steps 1 --warmup 1 --legs prefill_7b --prefill-modes ${PREFILL_MODES:-none,fused} --cpu-baseline-seconds 0 ;;
    pytestall) step pytest_gpu 1200 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
    bench)  step bench 600 python bench.py ${BENCH_ARGS:-} ;;
    gpucount) step gpucount 120 python -c "import bench, json; print(json.dumps({'visible_gpu_count': bench.visible_gpu_count()}))" ;;
    prof)   step rocprof 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 1 --legs none --cpu-baseline-seconds 0 ;;
    pmc)    step pmc 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o fetch -- python3 bench.py --steps 2 --warmup 1 --legs none --cpu-baseline-seconds 0 ;;
    shard1) step shard1 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --sharded --steps 3 --warmup 1 --legs none --cpu-baseline-seconds 0 ;;
    gpushard) step gpushard 900 python -m pytest tests/test_gpu_shard.py -q -p no:cacheprovider ;;
    qk) step qk 900 python -m pytest tests/test_gpu_qk.py -q -p no:cacheprovider ;;
    benchqk) step benchqk 900 python bench.py --importance qk --dtype float16 --steps 5 --warmup 2 ;;
    profqk) step rocprofqk 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profqk -o run -- python3 bench.py --importance qk --dtype float16 --steps 3 --warmup 1 ;;
    pmcw)   step pmcw 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw -o write -- python3 bench.py --steps 2 --warmup 1 --legs none --cpu-baseline-seconds 0 ;;
  esac
done
