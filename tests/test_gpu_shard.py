"""GPU: the sequence-shard entry points of the C ABI (rtkv_attention_aggregation_shard,
rtkv_finalize_select, rtkv_shard_ranges, rtkv_quantize_rows_shard) on one device.

N ranks are simulated one after another on cuda:0 (no collective needed: the test concatenates
the per-rank A itself and copies the rank byte ranges where the exchange would).  The union of the
ranks' outputs must equal the fused single-GPU rtkv_compress_layer output byte for byte, and each
rank's local dequantized rows must equal its slice of the single-GPU K'/V'."""
import numpy as np
import pytest
import torch

import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")


def _dev(a, dtype):
    if dtype == "float32":
        return torch.from_numpy(np.ascontiguousarray(a)).cuda()
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).cuda().view(getattr(torch, dtype))


@pytest.mark.parametrize("dtype,S_total,world,H,D,ratio", [
    ("float16", 4096, 2, 32, 128, 0.6),
    ("float16", 8192, 4, 32, 128, 0.4),
    ("bfloat16", 3000, 3, 8, 64, 0.8),     # P = 128, S_total*P not a multiple of 32 per shard boundary
    ("float32", 1500, 5, 4, 64, 0.3),
    ("float16", 640, 8, 4, 32, 0.05),      # tiny budget: the top-10% fallback across shards
    ("float16", 32768, 2, 8, 64, 0.5),
    ("float32", 65536, 4, 4, 128, 0.4),     # the one-launch K2 at its 64-workgroup limit
    ("float16", 81920, 8, 4, 64, 0.6),      # S_total above it: the pipeline K2 + the ranges kernel
    ("bfloat16", 8192, 4, 8, 64, -1.0),     # quantization only (RTKV_NO_SELECTION): the quant-only K2
    ("float16", 640, 1, 4, 32, 0.3),        # one rank
])
@pytest.mark.parametrize("fused", [False, True], ids=["separate", "fused"])
def test_shards_union_equals_single_gpu(dtype, S_total, world, H, D, ratio, fused):
    """The union of N simulated ranks equals the single-GPU layer byte for byte.  separate: the stage calls
    one by one (K1, finalize, ranges, K4); fused: the driver's calls — K1 that also clears the layer's
    selection scratch (rtkv_attention_aggregation_shard_ws), finalize + rank table in one call
    (rtkv_finalize_select_shard, scratch_zeroed = 1), then the split-row K4 over the rank's own rows."""
    import rtkv
    from rtkv import _lib as L
    from rtkv.sharded import HipShardStages, ShardBuffers
    F = H * D
    P = rtkv.prompt_length(S_total)
    K, V = synth.kv(77, 1, S_total, F, dtype)
    W = synth.attention_slice(77, 1, H, S_total, P, dtype)
    Kd, Vd, Wd = _dev(K, dtype), _dev(V, dtype), _dev(W, dtype)
    cfg = rtkv.CompressionConfig(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25, num_hidden_layers=1,
                                 layer_weights=[1.0], high_precision_bits=8, medium_precision_bits=4,
                                 low_precision_bits=2)
    flags = L.EMIT_DEQUANT | L.EMIT_PACKED | (L.NO_SELECTION if ratio < 0 else 0)
    params = rtkv.params_from_config(cfg, 0, P, abs(ratio), flags)
    bits = (2, 4, 8)
    # single GPU reference run
    ref = rtkv.LayerBuffers(1, S_total, F, Kd.dtype, "cuda", bits)
    ws = rtkv.Workspace("cuda")
    res = rtkv.compress_layer(Kd, Vd, Wd, params, ref, ws)
    st = res.stats()
    k_ref, v_ref = res.kv()
    # shards
    S_local = -(-S_total // world)
    if S_local * world != S_total:
        pytest.skip("uneven shards are not a configuration of the sharded path")
    stages = HipShardStages("cuda")
    A = torch.empty(1, S_total, dtype=torch.float32, device="cuda")
    for j in range(world):
        sl = slice(j * S_local, (j + 1) * S_local)
        stages.aggregate(Wd[:, :, sl], P, j * S_local, S_total, A[:, sl])
    bufs = [ShardBuffers(1, S_local, world, F, Kd.dtype, "cuda", bits) for _ in range(world)]
    for j in range(world):
        sl = slice(j * S_local, (j + 1) * S_local)
        if fused:  # rank j's K1 again (the same A rows), now clearing the scratch its finalize uses
            bufs[j].g.stats.fill_(0x5A)  # must be cleared by the K1 call
            stages.aggregate(Wd[:, :, sl], P, j * S_local, S_total, A[:, sl], params=params, bufs=bufs[j])
            stages.finalize_ranges(A, L.TORCH_DTYPE_CODE[Wd.dtype], params, bufs[j], world, zeroed=True)
        else:
            stages.finalize(A, L.TORCH_DTYPE_CODE[Wd.dtype], params, bufs[j])
            stages.ranges(bufs[j], world)
        stages.quantize(Kd[:, sl].contiguous(), Vd[:, sl].contiguous(), "bsf", j * S_local, j, world, params, bufs[j])
    torch.cuda.synchronize()
    n = st.max_kept
    tot = st.total_packed_bytes
    rg = bufs[0].ranges.cpu()
    assert int(rg[0, -1, 0]) == n and int(rg[0, -1, 1]) == tot
    for j in range(world):  # replicated selection
        g = bufs[j].g
        assert torch.equal(g.scores, ref.scores)
        assert torch.equal(g.labels, ref.labels)
        assert torch.equal(g.mask, ref.mask)
        assert torch.equal(g.kept_index[:, :n], ref.kept_index[:, :n])
        assert torch.equal(g.row_offset[:, :n], ref.row_offset[:, :n])
        assert torch.equal(bufs[j].ranges.cpu(), rg)
    pk = torch.zeros_like(ref.packed_k)
    pv = torch.zeros_like(ref.packed_v)
    sz = torch.zeros_like(ref.scale_zp)
    for j in range(world):  # what the exchange assembles
        r0, r1 = int(rg[0, j, 0]), int(rg[0, j + 1, 0])
        b0, b1 = int(rg[0, j, 1]), int(rg[0, j + 1, 1])
        g = bufs[j].g
        pk[b0:b1] = g.packed_k[b0:b1]
        pv[b0:b1] = g.packed_v[b0:b1]
        sz[:, r0:r1] = g.scale_zp[:, r0:r1]
        assert torch.equal(bufs[j].k_local[:, : r1 - r0], k_ref[:, r0:r1]), f"rank {j} local K'"
        assert torch.equal(bufs[j].v_local[:, : r1 - r0], v_ref[:, r0:r1]), f"rank {j} local V'"
    assert torch.equal(pk[:tot], ref.packed_k[:tot])
    assert torch.equal(pv[:tot], ref.packed_v[:tot])
    assert torch.equal(sz[:, :n], ref.scale_zp[:, :n])


@pytest.mark.parametrize("dtype,S_total,world,H,Hkv,ratio", [
    ("float16", 4096, 2, 32, 32, 0.6),
    ("bfloat16", 3072, 3, 16, 4, 0.5),   # GQA
])
def test_fused_mode_shards_union_equals_single_gpu(dtype, S_total, world, H, Hkv, ratio):
    """Fused importance mode on sequence shards (the prompt keys as rank 0 would broadcast them, each
    rank's A from its own Q rows and lse with row0): the per-rank A concatenates to the single-GPU
    rtkv_importance_qk_lse A bit for bit (64-row blocks line up), and the union of the ranks' outputs
    equals the fused single-GPU rtkv_compress_layer_qk output byte for byte."""
    import rtkv
    from rtkv import _lib as L
    from rtkv.sharded import HipShardStages, ShardBuffers
    D = 128
    F = Hkv * D
    P = rtkv.prompt_length(S_total)
    td = getattr(torch, dtype)
    g = torch.Generator(device="cuda").manual_seed(S_total)
    Kd = torch.randn(1, S_total, F, device="cuda", generator=g).to(td)
    Vd = torch.randn(1, S_total, F, device="cuda", generator=g).to(td)
    Q = torch.randn(1, H, S_total, D, device="cuda", generator=g).to(td)
    lse = rtkv.attention_lse(Q, Kd, k_layout="bsf")
    cfg = rtkv.CompressionConfig(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25, num_hidden_layers=1,
                                 layer_weights=[1.0], high_precision_bits=8, medium_precision_bits=4,
                                 low_precision_bits=2)
    params = rtkv.params_from_config(cfg, 0, P, ratio, L.EMIT_DEQUANT | L.EMIT_PACKED)
    bits = (2, 4, 8)
    ref = rtkv.LayerBuffers(1, S_total, F, td, "cuda", bits)
    res = rtkv.compress_layer_qk(Kd, Vd, Q, lse, params, ref, rtkv.Workspace("cuda"))
    st = res.stats()
    k_ref, v_ref = res.kv()
    A_ref = rtkv.importance_qk_lse(Q, Kd, lse, P)
    S_local = S_total // world
    stages = HipShardStages("cuda")
    kp = Kd[:, :P].contiguous()  # what rank 0 broadcasts
    A = torch.empty(1, S_total, dtype=torch.float32, device="cuda")
    for j in range(world):
        sl = slice(j * S_local, (j + 1) * S_local)
        A_loc = torch.empty(1, S_local, dtype=torch.float32, device="cuda")
        stages.aggregate_qk(Q[:, :, sl].contiguous(), kp, lse[:, :, sl].contiguous(), P, j * S_local, True, A_loc)
        A[:, sl] = A_loc
    assert torch.equal(A, A_ref)
    bufs = [ShardBuffers(1, S_local, world, F, td, "cuda", bits) for _ in range(world)]
    for j in range(world):
        stages.finalize(A, L.F32, params, bufs[j])
        stages.ranges(bufs[j], world)
        sl = slice(j * S_local, (j + 1) * S_local)
        stages.quantize(Kd[:, sl].contiguous(), Vd[:, sl].contiguous(), "bsf", j * S_local, j, world, params, bufs[j])
    torch.cuda.synchronize()
    n, tot = st.max_kept, st.total_packed_bytes
    rg = bufs[0].ranges.cpu()
    assert int(rg[0, -1, 0]) == n and int(rg[0, -1, 1]) == tot
    pk = torch.zeros_like(ref.packed_k)
    for j in range(world):
        g_ = bufs[j].g
        assert torch.equal(g_.kept_index[:, :n], ref.kept_index[:, :n])
        r0, r1 = int(rg[0, j, 0]), int(rg[0, j + 1, 0])
        b0, b1 = int(rg[0, j, 1]), int(rg[0, j + 1, 1])
        pk[b0:b1] = g_.packed_k[b0:b1]
        assert torch.equal(bufs[j].k_local[:, : r1 - r0], k_ref[:, r0:r1])
        assert torch.equal(bufs[j].v_local[:, : r1 - r0], v_ref[:, r0:r1])
    assert torch.equal(pk[:tot], ref.packed_k[:tot])


def test_rtkv_collectives_single_rank():
    """The C ABI's RCCL path (include/rtkv.h rtkv_comm_* / rtkv_allgather_rows / rtkv_allgather_packed,
    driven by ShardedPrefillCompressor(collectives='rtkv')) on a one-rank group: the communicator is
    made from a broadcast id, A goes through rtkv_allgather_rows, the exchange through
    rtkv_allgather_packed, and the layer equals the single-GPU result byte for byte.  (More ranks need
    more GPUs: the multi-rank exchange is the one rtkv/sharded.py's torch path runs, over the same
    rank byte ranges.)"""
    import os
    import socket
    import torch.distributed as dist
    import rtkv
    from rtkv.comm import RcclComm
    from rtkv.sharded import ShardedPrefillCompressor
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        comm = RcclComm.from_group()
        a_local = torch.randn(2, 300, device="cuda")
        a = torch.full((2, 300), float("nan"), device="cuda")
        comm.allgather_rows(a_local, a)
        torch.cuda.synchronize()
        assert torch.equal(a, a_local)
        comm.close()
        S, H, D, dtype = 2048, 8, 64, "float16"
        F, P = H * D, rtkv.prompt_length(S)
        K, V = synth.kv(91, 1, S, F, dtype)
        W = synth.attention_slice(91, 1, H, S, P, dtype)
        Kd, Vd, Wd = _dev(K, dtype), _dev(V, dtype), _dev(W, dtype)
        cfg = rtkv.CompressionConfig(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25,
                                     num_hidden_layers=1, layer_weights=[1.0], high_precision_bits=8,
                                     medium_precision_bits=4, low_precision_bits=2)
        outs = []
        for coll in ("torch", "rtkv"):
            comp = ShardedPrefillCompressor(cfg, collectives=coll, device="cuda")
            comp.enqueue_layer(Kd, Vd, Wd, 0)
            (sl,) = comp.exchange()
            torch.cuda.synchronize()
            g = sl.bufs.g
            n, tot = int(sl.ranges[0, -1, 0]), int(sl.ranges[0, -1, 1])
            outs.append((g.kept_index[:, :n].clone(), g.packed_k[:tot].clone(), g.packed_v[:tot].clone(),
                         g.scale_zp[:, :n].clone(), sl.bufs.k_local[:, :n].clone()))
        ref = rtkv.LayerBuffers(1, S, F, Kd.dtype, "cuda", (2, 4, 8))
        p = comp.params(0, S)
        res = rtkv.compress_layer(Kd, Vd, Wd, p, ref, rtkv.Workspace("cuda"))
        st = res.stats()
        k_ref, _ = res.kv()
        n, tot = st.max_kept, st.total_packed_bytes
        want = (ref.kept_index[:, :n], ref.packed_k[:tot], ref.packed_v[:tot], ref.scale_zp[:, :n], k_ref[:, :n])
        for got in outs:
            for x, y in zip(got, want):
                assert torch.equal(x, y)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,dtype,S_total,world,H,D,ratio", [
    ("cfg4", "float32", 65536, 8, 32, 128, 0.6),    # BASELINE configs[3]: 7B, S = 65536 over 8 ranks
    ("cfg4", "float16", 65536, 8, 32, 128, 0.4),
    ("cfg5", "float32", 32768, 8, 40, 128, 0.8),    # configs[4]: 13B shape (40 heads, F = 5120) over 8 ranks
    ("cfg5", "bfloat16", 32768, 8, 40, 128, 0.4),
])
def test_shards_union_equals_single_gpu_at_config_size(name, dtype, S_total, world, H, D, ratio):
    """The 8-way sequence-shard split at BASELINE's multi-GPU sizes (inputs generated on the device):
    S_total = 65536 takes the one-launch selection in rtkv_finalize_select (64 workgroups) on every rank, and
    rtkv_shard_ranges / rtkv_quantize_rows_shard split it 8 ways; the union equals the single-GPU
    rtkv_compress_layer byte for byte."""
    import rtkv
    from rtkv import _lib as L
    from rtkv.sharded import HipShardStages, ShardBuffers
    F = H * D
    P = rtkv.prompt_length(S_total)
    td = getattr(torch, dtype)
    g = torch.Generator(device="cuda").manual_seed(S_total + H)
    Kd = torch.randn(1, S_total, F, device="cuda", generator=g).to(td)
    Vd = torch.randn(1, S_total, F, device="cuda", generator=g).to(td)
    u = torch.rand(1, H, S_total, P, device="cuda", generator=g)
    Wd = (u * u) ** 2 + 1e-6
    Wd = Wd * (torch.arange(P, device="cuda")[None, :] <= torch.arange(S_total, device="cuda")[:, None])
    Wd = (Wd / Wd.sum(-1, keepdim=True) * torch.rand(1, H, S_total, 1, device="cuda", generator=g)).to(td)
    del u
    cfg = rtkv.CompressionConfig(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25, num_hidden_layers=1,
                                 layer_weights=[1.0], high_precision_bits=8, medium_precision_bits=4,
                                 low_precision_bits=2)
    params = rtkv.params_from_config(cfg, 0, P, ratio, L.EMIT_DEQUANT | L.EMIT_PACKED)
    bits = (2, 4, 8)
    ref = rtkv.LayerBuffers(1, S_total, F, td, "cuda", bits)
    res = rtkv.compress_layer(Kd, Vd, Wd, params, ref, rtkv.Workspace("cuda"))
    st = res.final_stats()
    k_ref, v_ref = res.kv()
    n, tot = st.max_kept, st.total_packed_bytes
    assert 0 < n < S_total
    S_local = S_total // world
    stages = HipShardStages("cuda")
    A = torch.empty(1, S_total, dtype=torch.float32, device="cuda")
    for j in range(world):
        sl = slice(j * S_local, (j + 1) * S_local)
        stages.aggregate(Wd[:, :, sl].contiguous(), P, j * S_local, S_total, A[:, sl])
    pk = torch.zeros_like(ref.packed_k)
    pv = torch.zeros_like(ref.packed_v)
    sz = torch.zeros_like(ref.scale_zp)
    bufs = ShardBuffers(1, S_local, world, F, td, "cuda", bits)  # one rank's buffers, reused rank after rank
    for j in range(world):
        stages.finalize(A, L.TORCH_DTYPE_CODE[td], params, bufs)
        stages.ranges(bufs, world)
        sl = slice(j * S_local, (j + 1) * S_local)
        stages.quantize(Kd[:, sl].contiguous(), Vd[:, sl].contiguous(), "bsf", j * S_local, j, world, params, bufs)
        torch.cuda.synchronize()
        gb = bufs.g
        assert torch.equal(gb.scores, ref.scores) and torch.equal(gb.mask, ref.mask)
        assert torch.equal(gb.kept_index[:, :n], ref.kept_index[:, :n])
        assert torch.equal(gb.row_offset[:, :n], ref.row_offset[:, :n])
        rg = bufs.ranges.cpu()
        assert int(rg[0, -1, 0]) == n and int(rg[0, -1, 1]) == tot
        r0, r1 = int(rg[0, j, 0]), int(rg[0, j + 1, 0])
        b0, b1 = int(rg[0, j, 1]), int(rg[0, j + 1, 1])
        assert r1 > r0, f"rank {j} keeps no row"
        pk[b0:b1] = gb.packed_k[b0:b1]
        pv[b0:b1] = gb.packed_v[b0:b1]
        sz[:, r0:r1] = gb.scale_zp[:, r0:r1]
        assert torch.equal(bufs.k_local[:, : r1 - r0], k_ref[:, r0:r1]), f"rank {j} local K'"
        assert torch.equal(bufs.v_local[:, : r1 - r0], v_ref[:, r0:r1]), f"rank {j} local V'"
    assert torch.equal(pk[:tot], ref.packed_k[:tot])
    assert torch.equal(pv[:tot], ref.packed_v[:tot])
    assert torch.equal(sz[:, :n], ref.scale_zp[:, :n])


def _golden_cases(prefix):
    from conftest import load_manifest
    return [c for c in load_manifest()["cases"] if c["name"].startswith(prefix)]


@pytest.mark.parametrize("case", _golden_cases("layer_cfg4_s65536"), ids=lambda c: c["name"])
def test_shards_union_matches_reference_golden_cfg4(case):
    """BASELINE configs[3] against the REFERENCE itself: the inputs of a reference-generated layer at
    S = 65536 (tests/golden/gen_golden.py runs RealTimePrefillCompressor.compress_layer_kv_cache on
    them) split over 8 simulated ranks.  Every rank's replicated scores / classes / mask equal the
    reference's, the ranks' local dequantized rows concatenated in rank order are the reference's
    K'/V' (sha256), and the assembled packed codes decode to the same bytes."""
    import rtkv
    from conftest import assert_matches, load_case
    from rtkv import _lib as L
    from rtkv.sharded import HipShardStages, ShardBuffers
    s = case["spec"]
    arrays = load_case(case)
    world, S_total, F, dt = 8, s["S"], s["Hkv"] * s["D"], s["dtype"]
    K, V = synth.kv(s["seed"], 1, S_total, F, dt)
    W = synth.attention_slice(s["seed"], 1, s["H"], S_total, s["P"], dt)
    Kd, Vd, Wd = _dev(K, dt), _dev(V, dt), _dev(W, dt)
    del K, V, W
    td = Kd.dtype
    pr = s["params"]
    cfg = rtkv.CompressionConfig(alpha=pr["alpha"], beta=pr["beta"], gamma=pr["gamma"], theta_h=pr["theta_h"],
                                 theta_m=pr["theta_m"], num_hidden_layers=s["L"], low_precision_bits=s["bits"][0],
                                 medium_precision_bits=s["bits"][1], high_precision_bits=s["bits"][2])
    assert cfg.layer_weights[s["layer"]] == s["layer_weight"]
    params = rtkv.params_from_config(cfg, s["layer"], s["P"], s["ratio"], L.EMIT_DEQUANT | L.EMIT_PACKED)
    bits = tuple(s["bits"])
    S_local = S_total // world
    stages = HipShardStages("cuda")
    A = torch.empty(1, S_total, dtype=torch.float32, device="cuda")
    for j in range(world):
        sl = slice(j * S_local, (j + 1) * S_local)
        stages.aggregate(Wd[:, :, sl].contiguous(), s["P"], j * S_local, S_total, A[:, sl])
    n = case["scalars"]["max_selected"]
    k_all = torch.empty(1, n, F, dtype=td, device="cuda")
    v_all = torch.empty(1, n, F, dtype=td, device="cuda")
    bufs = ShardBuffers(1, S_local, world, F, td, "cuda", bits)  # one rank's buffers, reused rank after rank
    pk = pv = sz = None
    for j in range(world):
        stages.finalize(A, L.TORCH_DTYPE_CODE[td], params, bufs)
        stages.ranges(bufs, world)
        sl = slice(j * S_local, (j + 1) * S_local)
        stages.quantize(Kd[:, sl].contiguous(), Vd[:, sl].contiguous(), "bsf", j * S_local, j, world, params, bufs)
        torch.cuda.synchronize()
        gb = bufs.g
        rg = bufs.ranges.cpu()
        assert int(rg[0, -1, 0]) == n
        if j == 0:  # the replicated global selection, against the reference
            assert_matches(case, "scores", gb.scores.cpu().numpy(), arrays)
            assert_matches(case, "labels", gb.labels.cpu().numpy(), arrays)
            assert_matches(case, "mask", gb.mask.cpu().numpy(), arrays)
            tot = int(rg[0, -1, 1])
            pk = torch.zeros(tot + 256, dtype=torch.uint8, device="cuda")  # decoders may read a line past the end
            pv = torch.zeros_like(pk)
            sz = torch.zeros(1, n, 4, dtype=torch.float32, device="cuda")
            kept_index, row_offset = gb.kept_index[:, :n].clone(), gb.row_offset[:, :n].clone()
            labels = gb.labels.clone()
        r0, r1 = int(rg[0, j, 0]), int(rg[0, j + 1, 0])
        b0, b1 = int(rg[0, j, 1]), int(rg[0, j + 1, 1])
        k_all[:, r0:r1] = bufs.k_local[:, : r1 - r0]
        v_all[:, r0:r1] = bufs.v_local[:, : r1 - r0]
        pk[b0:b1] = gb.packed_k[b0:b1]
        pv[b0:b1] = gb.packed_v[b0:b1]
        sz[:, r0:r1] = gb.scale_zp[:, r0:r1]

    def storage(t):
        t = t.cpu()
        return t.numpy() if t.dtype == torch.float32 else t.view(torch.int16).numpy().view(np.uint16)
    assert_matches(case, "k_out", storage(k_all), arrays)
    assert_matches(case, "v_out", storage(v_all), arrays)
    dk, dv = rtkv.unpack_layer(dict(codes_k=pk, codes_v=pv, row_offset=row_offset, scale_zp=sz, kept_index=kept_index,
                                    labels=labels, rows=[n], bits=bits, dtype=td, feature_dim=F))
    iv = torch.int32 if td == torch.float32 else torch.int16
    assert torch.equal(dk.view(iv), k_all.view(iv))
    assert torch.equal(dv.view(iv), v_all.view(iv))
