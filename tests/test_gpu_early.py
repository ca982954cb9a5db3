"""GPU: early statistics (rtkv_compress_layer_early).  The device publishes a layer's final counts to
host memory as soon as K2 has its thresholds; the drop-in path returns on them while K2's tail and K4
still run.  Every published field must equal the statistics the stream-synchronised read of the
device block gives after the layer (score_m2 / kept_score_sum excepted: they are read lazily), the
fallback and the pipeline path must report themselves as not published/incomplete, and the outputs
must not change."""
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


CASES = [  # dtype, B, S, H, D, ratio, expect: "complete" | "fallback" | "unpublished"
    ("float32", 1, 16384, 32, 128, 0.6, "complete"),
    ("float16", 1, 4096, 8, 64, 0.8, "complete"),
    ("bfloat16", 1, 777, 4, 64, 0.4, "complete"),
    ("float16", 1, 2000, 4, 32, 0.0001, "fallback"),    # U = 1 bit: nothing fits, the top-10% fallback
    ("float16", 2, 1024, 4, 32, 0.6, "unpublished"),    # B > 1: the pipeline K2
    ("float16", 1, 40000, 4, 32, 0.6, "complete"),      # 64 tokens per thread: the one-launch K2 up to S = 65536
    ("float16", 1, 70000, 4, 32, 0.6, "unpublished"),   # S > 65536: the pipeline K2
    ("float32", 1, 16384, 32, 128, 1.0, "quant"),       # RTKV_NO_SELECTION: the quantization-only K2
    ("bfloat16", 1, 3001, 4, 64, 1.0, "quant"),
]


@pytest.mark.parametrize("dtype,B,S,H,D,ratio,expect", CASES)
def test_early_stats_equal_the_final_block(dtype, B, S, H, D, ratio, expect):
    import rtkv
    from rtkv import _lib as L
    from rtkv.engine import EarlyStatsBuffer
    F = H * D
    P = rtkv.prompt_length(S)
    K, V = synth.kv(31 + S, B, S, F, dtype)
    W = synth.attention_slice(31 + S, B, H, S, P, dtype)
    Kd, Vd, Wd = _dev(K, dtype), _dev(V, dtype), _dev(W, dtype)
    cfg = rtkv.CompressionConfig(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25, num_hidden_layers=1,
                                 layer_weights=[1.0], high_precision_bits=8, medium_precision_bits=4,
                                 low_precision_bits=2)
    params = rtkv.params_from_config(cfg, 0, P, ratio, L.EMIT_DEQUANT | L.EMIT_PACKED |
                                     (L.NO_SELECTION if expect == "quant" else 0))
    ws = rtkv.Workspace("cuda")
    early = EarlyStatsBuffer()
    outs = []
    for use_early in (True, False):
        bufs = rtkv.LayerBuffers(B, S, F, Kd.dtype, "cuda", (2, 4, 8))
        res = rtkv.compress_layer(Kd, Vd, Wd, params, bufs, ws, early=early if use_early else None)
        st = res.stats()
        if use_early:
            published = res._early is not None
            assert published == (expect != "unpublished")
            if expect in ("complete", "quant"):
                assert np.isnan(st.score_m2) and np.isnan(st.batch[0]["kept_score_sum"])
        fin = res.final_stats()
        outs.append((st, fin, bufs))
    (st, fin, bufs_e), (_, ref, bufs_r) = outs
    for x in (st, fin):
        assert (x.max_kept, x.total_packed_bytes, x.error_flags) == (ref.max_kept, ref.total_packed_bytes,
                                                                      ref.error_flags)
        assert (x.score_sum, x.score_min, x.score_max) == (ref.score_sum, ref.score_min, ref.score_max)
        for a, b in zip(x.batch, ref.batch):
            for k in ("class_count", "kept", "kept_class", "cost_units", "packed_bytes", "fallback"):
                assert a[k] == b[k], k
    assert ref.batch[0]["fallback"] == (expect == "fallback")
    assert abs(fin.score_m2 - ref.score_m2) <= 1e-12 * max(1.0, abs(ref.score_m2))
    for a, b in zip(fin.batch, ref.batch):
        assert abs(a["kept_score_sum"] - b["kept_score_sum"]) <= 1e-12 * max(1.0, abs(b["kept_score_sum"]))
    n = ref.max_kept
    assert torch.equal(bufs_e.kept_index[:, :n], bufs_r.kept_index[:, :n])
    assert torch.equal(bufs_e.k_out[: B * n * F], bufs_r.k_out[: B * n * F])
    assert torch.equal(bufs_e.packed_v[: ref.total_packed_bytes], bufs_r.packed_v[: ref.total_packed_bytes])


@pytest.mark.parametrize("strict", [True, False])
def test_drop_in_returns_before_the_layer_finishes_and_stays_correct(strict):
    """The drop-in over consecutive layers (one early-stats buffer, rising sequence numbers): every
    layer's K'/V' and lazily read statistics equal a run that synchronises after each layer."""
    import rtkv
    S, H, D, dtype = 8192, 16, 128, "float16"
    F = H * D
    cfg = rtkv.CompressionConfig(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25, num_hidden_layers=6,
                                 high_precision_bits=8, medium_precision_bits=4, low_precision_bits=2)
    P = rtkv.prompt_length(S)
    ins = []
    for l in range(6):
        K, V = synth.kv(70 + l, 1, S, F, dtype)
        W = synth.attention_slice(70 + l, 1, H, S, P, dtype)
        ins.append((_dev(K, dtype), _dev(V, dtype), _dev(W, dtype)))
    ids = torch.zeros(1, S, dtype=torch.long, device="cuda")
    a, b = rtkv.RealTimePrefillCompressor(cfg, strict=strict), rtkv.RealTimePrefillCompressor(cfg)
    got = [a.compress_layer_kv_cache(K, V, W, ids, l) for l, (K, V, W) in enumerate(ins)]
    torch.cuda.synchronize()
    for l, (K, V, W) in enumerate(ins):
        k2, v2, info = b.compress_layer_kv_cache(K, V, W, ids, l)
        torch.cuda.synchronize()
        gk, gv, gi = got[l]
        assert gk.shape == k2.shape and torch.equal(gk.view(torch.int16), k2.view(torch.int16))
        assert torch.equal(gv.view(torch.int16), v2.view(torch.int16))
        for key in ("mean_score", "min_score", "max_score"):
            assert gi["importance_stats"][key] == info["importance_stats"][key]
        assert abs(gi["importance_stats"]["std_score"] - info["importance_stats"]["std_score"]) <= \
            1e-9 * abs(info["importance_stats"]["std_score"])
        ga = gi["propagation_info"]["selection_stats"]
        ra = info["propagation_info"]["selection_stats"]
        assert ga["selected_counts"] == ra["selected_counts"]
        assert np.allclose(ga["avg_importance"], ra["avg_importance"], rtol=1e-9, atol=0)
        assert np.array_equal(gi["quantization_info"]["bit_assignments"], info["quantization_info"]["bit_assignments"])
    assert a.get_overall_compression_stats()["total_layers_processed"] == 6


def test_withheld_selection_times_out_instead_of_hanging():
    """The one-launch K2's cross-workgroup waits are bounded (select_fast.hip poll_tagged): with the
    selection words withheld (RTKV_TEST_WITHHOLD_SELECTION) every waiting workgroup gives up after its
    poll bound, the kernel ends, the statistics carry RTKV_FLAG_SPIN_TIMEOUT and the host raises
    RTKV_ERR_TIMEOUT — both through the raw driver and through the drop-in (whose early publication is
    then marked incomplete, so it takes the synchronised statistics).  The next layer is unaffected."""
    import rtkv
    from rtkv import _lib as L
    from rtkv.engine import EarlyStatsBuffer
    S, H, D, dtype = 4096, 8, 64, "float16"
    F, P = H * D, rtkv.prompt_length(S)
    K, V = synth.kv(5, 1, S, F, dtype)
    W = synth.attention_slice(5, 1, H, S, P, dtype)
    Kd, Vd, Wd = _dev(K, dtype), _dev(V, dtype), _dev(W, dtype)
    cfg = rtkv.CompressionConfig(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25, num_hidden_layers=1,
                                 layer_weights=[1.0], high_precision_bits=8, medium_precision_bits=4,
                                 low_precision_bits=2)
    ok = rtkv.params_from_config(cfg, 0, P, 0.6, L.EMIT_DEQUANT | L.EMIT_PACKED)
    bad = rtkv.params_from_config(cfg, 0, P, 0.6, L.EMIT_DEQUANT | L.EMIT_PACKED | L.TEST_WITHHOLD_SELECTION)
    ws = rtkv.Workspace("cuda")
    for early in (None, EarlyStatsBuffer()):
        bufs = rtkv.LayerBuffers(1, S, F, Kd.dtype, "cuda", (2, 4, 8))
        res = rtkv.compress_layer(Kd, Vd, Wd, bad, bufs, ws, early=early)
        with pytest.raises(RuntimeError, match="RTKV_ERR_TIMEOUT"):
            res.stats()
        torch.cuda.synchronize()
        good = rtkv.LayerBuffers(1, S, F, Kd.dtype, "cuda", (2, 4, 8))
        st = rtkv.compress_layer(Kd, Vd, Wd, ok, good, ws, early=early).final_stats()
        assert st.error_flags == 0 and 0 < st.max_kept < S


def _lookback_inputs():
    import rtkv
    S, H, D, dtype = 4096, 8, 64, "float16"
    F, P = H * D, rtkv.prompt_length(S)
    K, V = synth.kv(6, 1, S, F, dtype)
    W = synth.attention_slice(6, 1, H, S, P, dtype)
    cfg = rtkv.CompressionConfig(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25, num_hidden_layers=4,
                                 high_precision_bits=8, medium_precision_bits=4, low_precision_bits=2)
    return S, F, P, cfg, _dev(K, dtype), _dev(V, dtype), _dev(W, dtype)


def test_lookback_timeout_after_the_early_publication_is_caught():
    """A hand-off that fails AFTER the early statistics are out (RTKV_TEST_WITHHOLD_LOOKBACK: workgroup 0
    never publishes its phase-3 counts): the early statistics are complete and clean, K4 then finds
    RTKV_FLAG_SPIN_TIMEOUT, writes NaN rows instead of codes and publishes the flag in the host mirror
    (final_flags), and the layer's final statistics raise RTKV_ERR_TIMEOUT."""
    import rtkv
    from rtkv import _lib as L
    from rtkv.engine import EarlyStatsBuffer, compress_layer_begin
    S, F, P, cfg, Kd, Vd, Wd = _lookback_inputs()
    p = rtkv.params_from_config(cfg, 0, P, 0.6, L.EMIT_DEQUANT | L.EMIT_PACKED | L.TEST_WITHHOLD_LOOKBACK)
    ws, early = rtkv.Workspace("cuda"), EarlyStatsBuffer()
    bufs = rtkv.LayerBuffers(1, S, F, Kd.dtype, "cuda", (2, 4, 8), outputs=False)
    res = compress_layer_begin(Kd, Vd, Wd, p, bufs, ws, early)
    with pytest.raises(RuntimeError, match=r"finish\(\) has not run"):
        ws.get(1, S)  # the workspace belongs to the pending layer
    st = res.stats()  # the early publication: complete, no flag yet
    assert res._early is not None and st.error_flags == 0 and 0 < st.max_kept < S
    res.finish()
    torch.cuda.synchronize()
    assert ws.pending is None
    assert res.final_flags() & L.FLAG_SPIN_TIMEOUT
    k, v = res.kv()
    assert torch.isnan(k.float()).all() and torch.isnan(v.float()).all()
    with pytest.raises(RuntimeError, match="RTKV_ERR_TIMEOUT"):
        res.final_stats()


def test_strict_drop_in_raises_a_late_timeout_in_the_failing_layer():
    """strict (the default): the call whose selection fails after the early statistics raises itself,
    so the reference caller's try/except (modified_llama.py:144-149) falls back for THAT layer: its
    uncompressed K/V are used, nothing NaN reaches attention, layer_states holds only the good layers
    and the next layers compress normally."""
    import rtkv
    from rtkv import _lib as L
    S, F, P, cfg, Kd, Vd, Wd = _lookback_inputs()
    ids = torch.zeros(1, S, dtype=torch.long, device="cuda")
    comp = rtkv.RealTimePrefillCompressor(cfg, strict=True)
    assert rtkv.RealTimePrefillCompressor(cfg).strict  # the default

    def caller(layer_idx):
        """modified_llama.py:102-149 in outline: compress, or print and keep the full K/V on any error."""
        try:
            k, v, _ = comp.compress_layer_kv_cache(Kd, Vd, Wd, ids, layer_idx)
            return k, v, False
        except Exception as e:  # noqa: BLE001 — the reference's catch-all
            print(f"Compression failed for layer {layer_idx}: {e}")
            return Kd, Vd, True

    outs = []
    for layer in range(4):
        comp._test_flags = L.TEST_WITHHOLD_LOOKBACK if layer == 1 else 0
        outs.append(caller(layer))
    comp._test_flags = 0
    torch.cuda.synchronize()
    assert [o[2] for o in outs] == [False, True, False, False]
    assert outs[1][0] is Kd
    for k, v, _ in outs:
        assert not torch.isnan(k.float()).any() and not torch.isnan(v.float()).any()
    assert sorted(comp.layer_states) == [0, 2, 3]
    ref = rtkv.RealTimePrefillCompressor(cfg, strict=False)
    r2, _, _ = ref.compress_layer_kv_cache(Kd, Vd, Wd, ids, 2)
    torch.cuda.synchronize()
    assert torch.equal(outs[2][0].view(torch.int16), r2.view(torch.int16))
    assert comp.get_overall_compression_stats()["total_layers_processed"] == 3


def test_non_strict_late_timeout_of_the_last_layer_raises_at_reset():
    """strict=False: a failing LAST layer of a forward must not vanish with reset_compression_state()
    (ADVICE r4): reset clears the state and then raises; verify_pending_layers() raises the same way
    before any reset."""
    import rtkv
    from rtkv import _lib as L
    S, F, P, cfg, Kd, Vd, Wd = _lookback_inputs()
    ids = torch.zeros(1, S, dtype=torch.long, device="cuda")
    for hook in ("reset", "verify"):
        comp = rtkv.RealTimePrefillCompressor(cfg, strict=False)
        comp.compress_layer_kv_cache(Kd, Vd, Wd, ids, 0)
        comp._test_flags = L.TEST_WITHHOLD_LOOKBACK
        comp.compress_layer_kv_cache(Kd, Vd, Wd, ids, 1)  # returns on its clean early statistics
        comp._test_flags = 0
        with pytest.raises(RuntimeError, match="layer 1"):
            comp.reset_compression_state() if hook == "reset" else comp.verify_pending_layers()
        if hook == "reset":
            assert comp.layer_states == {} and comp.importance_tracker.layer_scores == {}
        else:
            assert sorted(comp.layer_states) == [0]
        comp.reset_compression_state()  # nothing pending any more
        torch.cuda.synchronize()


def test_drop_in_reports_a_late_timeout_at_the_next_call():
    """strict=False: the drop-in returns on the early statistics; a layer whose selection failed after
    them is reported by the next call on the device (and by get_overall_compression_stats) from K4's
    host flags, without a stream sync per layer, and the layer is dropped from layer_states.  The
    layers after it are unaffected.  (A documented deviation from the reference's synchronous call,
    INTEGRATION.md §4; strict=True, the default, raises in the failing layer.)"""
    import rtkv
    S, F, P, cfg, Kd, Vd, Wd = _lookback_inputs()
    ids = torch.zeros(1, S, dtype=torch.long, device="cuda")
    from rtkv import _lib as L
    comp = rtkv.RealTimePrefillCompressor(cfg, strict=False)
    k0, v0, _ = comp.compress_layer_kv_cache(Kd, Vd, Wd, ids, 0)  # good layer
    comp._test_flags = L.TEST_WITHHOLD_LOOKBACK
    k1, v1, _ = comp.compress_layer_kv_cache(Kd, Vd, Wd, ids, 1)  # returns on its (clean) early statistics
    comp._test_flags = 0
    with pytest.raises(RuntimeError, match="layer 1"):
        comp.compress_layer_kv_cache(Kd, Vd, Wd, ids, 2)
    torch.cuda.synchronize()
    assert torch.isnan(k1.float()).all()
    k3, v3, _ = comp.compress_layer_kv_cache(Kd, Vd, Wd, ids, 3)
    torch.cuda.synchronize()
    ref = rtkv.RealTimePrefillCompressor(cfg, strict=False)
    r3, _, _ = ref.compress_layer_kv_cache(Kd, Vd, Wd, ids, 3)
    assert torch.equal(k3.view(torch.int16), r3.view(torch.int16))
    assert sorted(comp.layer_states) == [0, 3]
    assert comp.get_overall_compression_stats()["total_layers_processed"] == 2
    # the same through get_overall_compression_stats when the failing layer is the last one
    comp._test_flags = L.TEST_WITHHOLD_LOOKBACK
    comp.compress_layer_kv_cache(Kd, Vd, Wd, ids, 2)
    comp._test_flags = 0
    with pytest.raises(RuntimeError, match="layer 2"):
        comp.get_overall_compression_stats()


def test_finish_with_undersized_outputs_writes_nothing():
    """rtkv_compress_layer_finish with buffers smaller than the layer's published sizes (out_rows below
    S'_max, or packed_capacity below the code bytes): K4 writes nothing, flags
    RTKV_FLAG_OUTPUT_OVERFLOW in the statistics and in the host mirror."""
    import ctypes
    import rtkv
    from rtkv import _lib as L
    from rtkv.engine import EarlyStatsBuffer, compress_layer_begin
    S, F, P, cfg, Kd, Vd, Wd = _lookback_inputs()
    p = rtkv.params_from_config(cfg, 0, P, 0.6, L.EMIT_DEQUANT | L.EMIT_PACKED)
    for short in ("rows", "bytes"):
        ws, early = rtkv.Workspace("cuda"), EarlyStatsBuffer()
        bufs = rtkv.LayerBuffers(1, S, F, Kd.dtype, "cuda", (2, 4, 8), outputs=False)
        res = compress_layer_begin(Kd, Vd, Wd, p, bufs, ws, early)
        st = res.stats()
        n, nb = st.max_kept, st.total_packed_bytes
        rows = n - 1 if short == "rows" else n
        cap = nb if short == "rows" else nb - 1
        kv = torch.full((2, 1, n, F), 7.0, dtype=Kd.dtype, device="cuda")  # room for n rows, declared `rows`
        codes = torch.full((2, nb + 256), 0xAB, dtype=torch.uint8, device="cuda")
        out = res._out
        out.k_out_dev, out.v_out_dev = kv[0].data_ptr(), kv[1].data_ptr()
        out.packed_k_dev, out.packed_v_dev = codes[0].data_ptr(), codes[1].data_ptr()
        out.packed_capacity = cap
        L.check(L.lib().rtkv_compress_layer_finish(ctypes.byref(res._kd), ctypes.byref(p), ctypes.byref(out), rows,
                                                   ws.buf.data_ptr(), ws.buf.numel(), L.stream_ptr(Kd.device),
                                                   early.ptr, res._seq), "finish")
        ws.pending = None
        torch.cuda.synchronize()
        assert early.final_flags(res._seq) & L.FLAG_OUTPUT_OVERFLOW
        assert bool((kv == 7.0).all()) and bool((codes == 0xAB).all())
        with pytest.raises(RuntimeError, match="RTKV_FLAG_OUTPUT_OVERFLOW"):
            res.final_stats()


def test_prefetch_and_start_event_leave_the_outputs_unchanged():
    """The drop-in's kept-row prefetch (loads only, any size, a no-op for B > 1) and the begin call's
    optional start event do not change a byte of the layer's outputs; the event is recorded (its
    elapsed time to the completion event is positive)."""
    import rtkv
    from rtkv import _lib as L
    from rtkv.engine import EarlyStatsBuffer, compress_layer_begin
    S, F = 2048, 1024
    g = torch.Generator(device="cuda").manual_seed(3)
    P = rtkv.prompt_length(S)
    cfg = rtkv.CompressionConfig(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25, num_hidden_layers=4,
                                 high_precision_bits=8, medium_precision_bits=4, low_precision_bits=2)
    outs = []
    for B, pf in ((1, 0), (1, 1 << 40), (2, 0), (2, 1 << 40)):
        K = torch.randn(B, S, F, device="cuda", generator=g)
        V = torch.randn(B, S, F, device="cuda", generator=g)
        W = torch.rand(B, 8, S, P, device="cuda", generator=g)
        if pf:  # same inputs as the previous case
            K, V, W = prev
        prev = (K, V, W)
        comp = rtkv.RealTimePrefillCompressor(cfg)
        comp.prefetch_bytes = pf
        ids = torch.zeros(B, S, dtype=torch.long, device="cuda")
        k, v, info = comp.compress_layer_kv_cache(K, V, W, ids, 1)
        outs.append((k.clone(), v.clone(), info["packed"]["codes_k"].clone(), info["packed"]["codes_v"].clone()))
    for a, b in ((0, 1), (2, 3)):
        for x, y in zip(outs[a], outs[b]):
            assert torch.equal(x.view(torch.uint8) if x.dtype != torch.uint8 else x,
                               y.view(torch.uint8) if y.dtype != torch.uint8 else y)
    # the start event: recorded by rtkv_compress_layer_begin right before K1
    K, V, W = prev[0][:1].contiguous(), prev[1][:1].contiguous(), prev[2][:1].contiguous()
    p = rtkv.params_from_config(cfg, 1, P, 0.6, L.EMIT_DEQUANT | L.EMIT_PACKED)
    bufs = rtkv.LayerBuffers(1, S, F, torch.float32, "cuda", (2, 4, 8), outputs=False)
    ev = torch.cuda.Event(enable_timing=True)
    ev.record()  # creates the hipEvent_t (torch makes it at the first record)
    early = EarlyStatsBuffer()
    res = compress_layer_begin(K, V, W, p, bufs, rtkv.Workspace("cuda"), early, start_event=ev.cuda_event)
    res.finish()
    res.done.synchronize()
    end = torch.cuda.Event(enable_timing=True)
    end.record()
    end.synchronize()
    assert ev.elapsed_time(end) > 0 and 0 < res.device_seconds() < ev.elapsed_time(end) / 1e3 + 1e-5


def test_finish_exact_rejects_oversized_outputs():
    """RTKV_FINISH_EXACT (the drop-in's flag): buffers LARGER than the device statistics give — what a
    torn or stale read of the early line would produce (an S' or byte count from another layer) — are
    flagged RTKV_FLAG_OUTPUT_OVERFLOW and nothing is written; the exact sizes pass (advisor, round 5)."""
    import ctypes
    import rtkv
    from rtkv import _lib as L
    from rtkv.engine import EarlyStatsBuffer, compress_layer_begin
    S, F, P, cfg, Kd, Vd, Wd = _lookback_inputs()
    p = rtkv.params_from_config(cfg, 0, P, 0.6, L.EMIT_DEQUANT | L.EMIT_PACKED | L.FINISH_EXACT)
    for case in ("exact", "rows", "bytes"):
        ws, early = rtkv.Workspace("cuda"), EarlyStatsBuffer()
        bufs = rtkv.LayerBuffers(1, S, F, Kd.dtype, "cuda", (2, 4, 8), outputs=False)
        res = compress_layer_begin(Kd, Vd, Wd, p, bufs, ws, early)
        st = res.stats()
        n, nb = st.max_kept, st.total_packed_bytes
        rows = n + 1 if case == "rows" else n
        cap = (nb + 255) // 256 * 256 + (256 if case == "bytes" else 0)
        kv = torch.full((2, 1, n + 1, F), 7.0, dtype=Kd.dtype, device="cuda")
        codes = torch.full((2, cap), 0xAB, dtype=torch.uint8, device="cuda")
        out = res._out
        out.k_out_dev, out.v_out_dev = kv[0].data_ptr(), kv[1].data_ptr()
        out.packed_k_dev, out.packed_v_dev = codes[0].data_ptr(), codes[1].data_ptr()
        out.packed_capacity = cap
        L.check(L.lib().rtkv_compress_layer_finish(ctypes.byref(res._kd), ctypes.byref(p), ctypes.byref(out), rows,
                                                   ws.buf.data_ptr(), ws.buf.numel(), L.stream_ptr(Kd.device),
                                                   early.ptr, res._seq), "finish")
        ws.pending = None
        torch.cuda.synchronize()
        if case == "exact":
            assert early.final_flags(res._seq) == 0
            assert not bool((kv[:, :, :n] == 7.0).all())
            res.final_stats()
        else:
            assert early.final_flags(res._seq) & L.FLAG_OUTPUT_OVERFLOW
            assert bool((kv == 7.0).all()) and bool((codes == 0xAB).all())
            with pytest.raises(RuntimeError, match="RTKV_FLAG_OUTPUT_OVERFLOW"):
                res.final_stats()
