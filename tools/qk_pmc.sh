# Counter passes for the fused-mode MFMA kernels: LDS traffic, wave stall shares, VALU/MFMA activity,
# one rocprofv3 pass per counter set (8 SQ counters at most per pass).
#   bash tools/qk_pmc.sh            K1' (bench.py --importance qk, 4 layers)
#   PROG=lse bash tools/qk_pmc.sh   attn_lse_kernel (tools/lse_bench.py)
#   PROG=k4 bash tools/qk_pmc.sh    quant_rows_kernel, fp16 packed-only
set -e
mkdir -p gpurun_out/qkpmc
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
if [ "${PROG:-qk}" = lse ]; then
  CMD="$R/tools/lse_bench.py"
elif [ "${PROG:-qk}" = k4 ]; then  # K4 at f16, packed codes only
  CMD="$R/bench.py --dtype float16 --no-dequant --layers 4 --steps 2 --warmup 1 --legs none --cpu-baseline-seconds 0 --streams 1"
elif [ "${PROG:-qk}" = k4f32 ]; then  # K4 at fp32, dequant + packed (the headline workload)
  CMD="$R/bench.py --layers 4 --steps 2 --warmup 1 --legs none --cpu-baseline-seconds 0 --streams 1"
elif [ "${PROG:-qk}" = k4f32p ]; then  # K4 at fp32, packed codes only
  CMD="$R/bench.py --no-dequant --layers 4 --steps 2 --warmup 1 --legs none --cpu-baseline-seconds 0 --streams 1"
else
  CMD="$R/bench.py --importance qk --dtype float16 --layers 4 --steps 2 --warmup 1 --legs none --cpu-baseline-seconds 0 --streams 1"
fi
n=0
for P in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
         "SQ_WAVES SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM GRBM_GUI_ACTIVE"; do
  n=$((n + 1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/qkpmc -o ${PROG:-qk}$n -- python3 $CMD > $R/gpurun_out/qkpmc/${PROG:-qk}$n.log 2>&1
done
