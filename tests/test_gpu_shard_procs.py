"""GPU, several processes: the sequence-sharded prefill with the HIP shard stages in SEPARATE processes
that share the one GPU, over a gloo group whose exchanges are staged through
host memory (ShardedPrefillCompressor(collectives='host')).  Each rank (tests/shard_procs_worker.py)
compares what it holds after the exchange with the single-GPU rtkv_compress_layer of the whole
sequence, byte for byte; the parent only launches the ranks and checks that every one reports ok."""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,S_total,H,D,dtype,layers,B,mode,overlap", [
    (2, 8192, 32, 128, "float32", 2, 1, "w", 1),     # Llama-2-7B rows, the reference's fp32
    (2, 4096, 8, 128, "float16", 3, 2, "w", 0),      # B = 2: the pipeline selection, batch-row spans
    (2, 4096, 8, 128, "bfloat16", 2, 1, "qk", 1),    # fused importance mode: prompt keys broadcast from rank 0
    (4, 4096, 8, 64, "float16", 2, 1, "w", 1),       # four ranks on the one GPU
])
def test_hip_stages_in_separate_processes(world, S_total, H, D, dtype, layers, B, mode, overlap):
    _run_ranks(world, S_total, H, D, dtype, layers, B, mode, overlap, "host")


@pytest.mark.parametrize("coll", ["torch", "rtkv"])
@pytest.mark.parametrize("S_total,H,D,dtype,layers,B,mode,overlap", [
    (8192, 32, 128, "float32", 2, 1, "w", 1),
    (4096, 8, 128, "float16", 3, 2, "w", 0),      # B = 2: batch-row byte and scale/zp offsets
    (4096, 8, 128, "bfloat16", 2, 1, "qk", 1),
])
def test_rccl_collectives_two_gpus(S_total, H, D, dtype, layers, B, mode, overlap, coll):
    """Two ranks on two GPUs over RCCL: torch.distributed collectives and the C ABI's own
    (rtkv_comm_init / rtkv_allgather_rows / rtkv_allgather_packed on the exchange stream, beside the
    A all-gather communicator when overlap = 1): every rank's packed KV equals the single-GPU layer byte
    for byte.  Needs two devices; the one-GPU test box skips it (there RCCL cannot place two ranks)."""
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    _run_ranks(2, S_total, H, D, dtype, layers, B, mode, overlap, coll)


def _run_ranks(world, S_total, H, D, dtype, layers, B, mode, overlap, coll):
    port = _free_port()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "shard_procs_worker.py"), str(r), str(world),
                               str(port), str(S_total), str(H), str(D), dtype, str(layers), str(B), mode, str(overlap),
                               coll],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env, text=True)
             for r in range(world)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=240)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, (p, o) in enumerate(zip(procs, outs)):
        assert p.returncode == 0 and f"rank {r} ok" in o, f"rank {r} (rc={p.returncode}):\n{o[-4000:]}"
