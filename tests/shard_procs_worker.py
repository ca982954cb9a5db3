"""One rank of tests/test_gpu_shard_procs.py (run as its own process; not collected by pytest).

    python tests/shard_procs_worker.py RANK WORLD PORT S_TOTAL H D DTYPE LAYERS B MODE OVERLAP [COLL]

Every rank drives rtkv.sharded.ShardedPrefillCompressor with the HIP stages (librtkv.so) on the
shared GPU, over a gloo group with the exchanges staged through host memory (COLL = 'host', the
default), or on its own GPU (cuda:RANK) over an RCCL group with COLL = 'torch' (torch.distributed) or
'rtkv' (the C ABI's rtkv_comm_* / rtkv_allgather_* collectives),
then checks what it holds after the exchange against the single-GPU rtkv_compress_layer of the whole
sequence, computed in this same process from the same seeded inputs: kept indices, row offsets,
packed K/V codes and scale/zero-point byte for byte, and its own dequantized rows."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(HERE, ".."), os.path.join(HERE, "..", "realtime-kv-cache-compression_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def inputs(l, B, S, H, D, td, qk):
    g = torch.Generator(device="cuda").manual_seed(1000 + l)
    F = H * D
    P = min(S // 5, 128)
    K = torch.randn(B, S, F, device="cuda", generator=g).to(td)
    V = torch.randn(B, S, F, device="cuda", generator=g).to(td)
    if qk:
        Q = torch.randn(B, H, S, D, device="cuda", generator=g).to(td)
        return K, V, Q, P
    u = torch.rand(B, H, S, P, device="cuda", generator=g)
    W = (u * u) ** 2 + 1e-6
    W = W * (torch.arange(P, device="cuda")[None, :] <= torch.arange(S, device="cuda")[:, None])
    W = (W / W.sum(-1, keepdim=True) * torch.rand(B, H, S, 1, device="cuda", generator=g)).to(td)
    return K, V, W, P


def main():
    rank, world, port, S_total, H, D = (int(x) for x in sys.argv[1:7])
    dtype, layers, B, mode, overlap = sys.argv[7], int(sys.argv[8]), int(sys.argv[9]), sys.argv[10], sys.argv[11] == "1"
    coll = sys.argv[12] if len(sys.argv) > 12 else "host"
    if coll == "host":
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world, init_method=f"tcp://127.0.0.1:{port}")
    else:  # one GPU per rank, RCCL
        torch.cuda.set_device(rank)
        dist.init_process_group("nccl", rank=rank, world_size=world, init_method=f"tcp://127.0.0.1:{port}",
                                device_id=torch.device("cuda", rank))
    import rtkv
    from rtkv.sharded import ShardedPrefillCompressor
    td = getattr(torch, dtype)
    cfg = rtkv.CompressionConfig(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25, high_precision_bits=8,
                                 medium_precision_bits=4, low_precision_bits=2, early_layer_ratio=0.8,
                                 middle_layer_ratio=0.6, later_layer_ratio=0.4, num_hidden_layers=layers)
    comp = ShardedPrefillCompressor(cfg, device=f"cuda:{torch.cuda.current_device()}", collectives=coll,
                                    overlap=overlap)
    assert type(comp.stages).__name__ == "HipShardStages"
    S_local = S_total // world
    sl = slice(rank * S_local, (rank + 1) * S_local)
    full = []
    for l in range(layers):
        K, V, X, P = inputs(l, B, S_total, H, D, td, mode == "qk")
        if mode == "qk":
            lse = rtkv.attention_lse(X, K, k_layout="bsf")
            comp.enqueue_layer_qk(K[:, sl].contiguous(), V[:, sl].contiguous(), X[:, :, sl].contiguous(),
                                  lse[:, :, sl].contiguous(), l)
            full.append((K, V, X, lse))
        else:
            comp.enqueue_layer(K[:, sl].contiguous(), V[:, sl].contiguous(), X[:, :, sl].contiguous(), l)
            full.append((K, V, X, None))
    out = comp.exchange()
    torch.cuda.synchronize()
    assert [s.layer_idx for s in out] == list(range(layers))
    for s in out:
        K, V, X, lse = full[s.layer_idx]
        p = comp.params(s.layer_idx, S_total)
        ref = rtkv.LayerBuffers(B, S_total, H * D, td, "cuda", (2, 4, 8))
        if mode == "qk":
            res = rtkv.compress_layer_qk(K, V, X, lse, p, ref, rtkv.Workspace("cuda"))
        else:
            res = rtkv.compress_layer(K, V, X, p, ref, rtkv.Workspace("cuda"))
        st = res.final_stats()
        g = s.bufs.g
        for b in range(B):
            n = st.batch[b]["kept"]
            assert s.kept(b) == n, (s.layer_idx, b, s.kept(b), n)
            assert torch.equal(g.kept_index[b, :n], ref.kept_index[b, :n]), "kept_index"
            assert torch.equal(g.row_offset[b, :n], ref.row_offset[b, :n]), "row_offset"
            assert torch.equal(g.scale_zp[b, :n], ref.scale_zp[b, :n]), "scale/zero-point"
        tot = st.total_packed_bytes
        assert torch.equal(g.packed_k[:tot], ref.packed_k[:tot]), "packed K"
        assert torch.equal(g.packed_v[:tot], ref.packed_v[:tot]), "packed V"
        # this rank's own dequantized rows = its slice of the single-GPU K'/V'
        kr = ref.k_out[: B * st.max_kept * H * D].view(B, st.max_kept, H * D)
        k_loc, _ = s.local_kv(rank)
        for b in range(B):
            r0, r1 = int(s.ranges[b, rank, 0]), int(s.ranges[b, rank + 1, 0])
            assert torch.equal(k_loc[b, : r1 - r0], kr[b, r0:r1]), "local K' rows"
    dist.barrier()
    dist.destroy_process_group()
    print(f"rank {rank} ok: {layers} layers, S_total={S_total}, world={world}, {dtype}, B={B}, mode={mode}, "
          f"collectives={coll}", flush=True)


if __name__ == "__main__":
    main()
