# Round-6 evidence batch: the fused-mode mismatch tests, the K2 phase timeline (tools/k2_probe) at
# S = 16384 / 4096 / 65536 (+ the sharded finalize's form: A without K1 partials), FETCH/WRITE PMC and
# kernel stats of the S = 65536 workload, and the MFMA counter passes (tools/mfma_pmc.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06f
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_fused_mismatch.py > $O/mismatch.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
for a in "16384 0.6" "4096 0.6" "65536 0.6" "65536 0.6 bench row"; do
  timeout -k 10 120 ./tools/k2_probe $a > $O/k2probe_$(echo $a | tr ' ' _).txt 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --seq 65536 --legs none --cpu-baseline-seconds 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $B --steps 3 --warmup 1 > $O/prof.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc -o fetch -- python3 $B --steps 2 --warmup 1 > $O/pmc.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw -o write -- python3 $B --steps 2 --warmup 1 > $O/pmcw.log 2>&1 || exit 1
cd $R
bash tools/mfma_pmc.sh
