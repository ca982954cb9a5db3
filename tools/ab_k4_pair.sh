# A/B of the paired packed-only K4 (RTKV_K4_PK_PAIR) on the f16 packed-only leg, then its parity tests
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-a}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k packed_only -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_pair_$T.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_pair_$T.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for p in 3 0; do
  RTKV_K4_PK_PAIR=$p timeout -k 10 300 python bench.py --legs f16_packed_only --steps 10 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/ab_${T}_pair${p}_r$r.json 2> gpurun_out/ab_${T}_pair${p}_r$r.err || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/ab_${T}_pair${p}_r$r.json').read().strip().splitlines()[-1]);l=d['legs']['f16_packed_only'];print('round',$r,'pair',$p,'ms',l['ms_per_step'],'K4',l['kernel_us_per_layer'],'frac',l['path_read_roofline_frac'])"
done; done
