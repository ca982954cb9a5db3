# MFMA evidence for the two MFMA kernels (attn_lse_kernel, qk_importance_kernel): rocprofv3 counter
# passes (each its own run) over tools/lse_bench.py and the fused-mode bench, summarised by
# tools/mfma_summary.py.  Utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (kernel duration x clock x 1024 SIMDs), clock checked <= 2.4 GHz.
set -e
mkdir -p gpurun_out/mfma
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
QK="$R/bench.py --importance qk --dtype float16 --layers 4 --steps 2 --warmup 1 --legs none --cpu-baseline-seconds 0"
# (QK_ENV: extra environment for the fused-mode runs, e.g. RTKV_QK_COAL=1 — exported, not a launcher hop)
[ -n "${QK_ENV:-}" ] && export $QK_ENV
# (SKIP_LSE=1: the fused-mode kernels only; EXTRA_PASS: one more counter pass, e.g. cache counters)
PASSES=("SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS")
[ -n "${EXTRA_PASS:-}" ] && PASSES+=("$EXTRA_PASS")
for P in "${PASSES[@]}"; do
  tag=$(echo $P | cut -c1-12 | tr -c 'A-Za-z0-9\n' _)
  [ -z "${SKIP_LSE:-}" ] && timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/mfma/lse -o $tag -- python3 $R/tools/lse_bench.py > $R/gpurun_out/mfma/lse_$tag.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/mfma/qk -o $tag -- python3 $QK > $R/gpurun_out/mfma/qk_$tag.log 2>&1
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/mfma/qk -o trace -- python3 $QK > $R/gpurun_out/mfma/qk_trace.log 2>&1
