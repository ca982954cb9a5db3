# decode: PMC passes (one counter group per run) over config 1 of tools/decode_bench.py
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp
P=$GRAFT_REPO_ROOT/tools/decode_bench.py
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_WAIT_ANY -d $GRAFT_REPO_ROOT/gpurun_out/pmc1 -o p --output-format csv -- python3 $P 1 20 > $GRAFT_REPO_ROOT/gpurun_out/pmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -d $GRAFT_REPO_ROOT/gpurun_out/pmc2 -o p --output-format csv -- python3 $P 1 20 > $GRAFT_REPO_ROOT/gpurun_out/pmc2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_IFETCH SQ_THREAD_CYCLES_VALU SQ_LEVEL_WAVES -d $GRAFT_REPO_ROOT/gpurun_out/pmc3 -o p --output-format csv -- python3 $P 1 20 > $GRAFT_REPO_ROOT/gpurun_out/pmc3.log 2>&1 || exit 1
