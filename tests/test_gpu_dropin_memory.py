"""GPU: what the drop-in (RealTimePrefillCompressor.compress_layer_kv_cache) allocates and retains.

The reference returns K'/V' of exactly S' rows (selective_propagation.py:214-232,
unified_compressor.py:170).  rtkv sizes them from the early statistics (rtkv_compress_layer_begin /
_finish), so a layer's K'/V' hold 2·B·S'·F elements, its packed codes exactly their bytes, and the
compressor's layer_states keep only per-token buffers and the packed codes: once the caller drops K'/V'
nothing pins them, and reset_compression_state() releases the rest."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")


def _round(n):  # the caching allocator's granule (memory_allocated counts rounded block sizes)
    return (n + 511) // 512 * 512


# A block the caching allocator hands out may exceed the request by up to 1 MiB (it does not split off
# a remainder of <= 1 MiB from a cached segment); two large allocations per layer (K'+V', the codes).
SLACK = 2 * (1 << 20) + 256 * 1024


@pytest.mark.parametrize("dtype", ["float16", "float32"])
def test_dropin_retains_exactly_the_kept_rows(dtype):
    import rtkv
    S, H, D, layers = 8192, 32, 128, 6
    F = H * D
    td = getattr(torch, dtype)
    esz = torch.tensor([], dtype=td).element_size()
    cfg = rtkv.CompressionConfig(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25, num_hidden_layers=layers,
                                 high_precision_bits=8, medium_precision_bits=4, low_precision_bits=2,
                                 early_layer_ratio=0.8, middle_layer_ratio=0.6, later_layer_ratio=0.4)
    g = torch.Generator(device="cuda").manual_seed(5)
    P = rtkv.prompt_length(S)
    ins = []
    for _ in range(layers):
        K = torch.randn(1, S, F, device="cuda", generator=g).to(td)
        V = torch.randn(1, S, F, device="cuda", generator=g).to(td)
        u = torch.rand(1, H, S, P, device="cuda", generator=g)
        W = ((u * u) ** 2 + 1e-6)
        W = (W / W.sum(-1, keepdim=True) * torch.rand(1, H, S, 1, device="cuda", generator=g)).to(td)
        ins.append((K, V, W))
    ids = torch.zeros(1, S, dtype=torch.long, device="cuda")
    comp = rtkv.RealTimePrefillCompressor(cfg)
    comp.compress_layer_kv_cache(*ins[0], ids, 0)  # workspace + early-stats buffer exist from here on
    comp.reset_compression_state()
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    kept = []
    for l, (K, V, W) in enumerate(ins):
        kept.append(comp.compress_layer_kv_cache(K, V, W, ids, l)[:2])
    torch.cuda.synchronize()
    grown = torch.cuda.memory_allocated() - base
    rows = [k.shape[1] for k, _ in kept]
    packed = [int(comp.layer_states[l]["packed"]["codes_k"].numel()) for l in range(layers)]
    meta = 34 * S + 4096  # per layer: scores, classes, mask, kept index, row offset, scale/zero-point, stats
    exact = sum(_round(2 * r * F * esz) + _round(2 * ((pb + 255) // 256 * 256)) + meta for r, pb in zip(rows, packed))
    assert all(0 < r < S for r in rows)
    assert grown <= exact + SLACK * layers, (grown, exact)
    # capacity-sized outputs (S rows of K'/V' and S rows of 8-bit codes per tensor) would not fit that bound
    assert exact + SLACK * layers < layers * (2 * S * F * esz + 2 * S * F)
    # the caller drops K'/V': nothing the compressor keeps pins them
    del kept
    torch.cuda.synchronize()
    held = torch.cuda.memory_allocated() - base
    assert held <= sum(_round(2 * ((pb + 255) // 256 * 256)) + meta for pb in packed) + SLACK * layers, held
    info = comp.layer_states[layers - 1]
    assert info["packed"]["codes_k"].numel() == packed[-1] and info["processing_time"] > 0
    del info  # (it references the layer's codes)
    comp.reset_compression_state()
    torch.cuda.synchronize()
    assert torch.cuda.memory_allocated() - base <= 256 * 1024


def test_device_processing_time_is_the_device_span_without_events():
    """device_processing_time is the layer's device time span stamped by the kernels themselves
    (rtkv_layer_times: the first K1 block's start to the last K4 workgroup's end on the 100 MHz
    real-time counter): positive, within the span of HIP events recorded around the call, and the call
    records no event of its own but the layer's completion."""
    import rtkv
    S, F, layers = 4096, 4096, 6
    cfg = rtkv.CompressionConfig(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25, num_hidden_layers=layers,
                                 high_precision_bits=8, medium_precision_bits=4, low_precision_bits=2)
    g = torch.Generator(device="cuda").manual_seed(9)
    P = rtkv.prompt_length(S)
    K = torch.randn(1, S, F, device="cuda", generator=g)
    V = torch.randn(1, S, F, device="cuda", generator=g)
    W = torch.rand(1, 32, S, P, device="cuda", generator=g)
    W = W / W.sum(-1, keepdim=True)
    ids = torch.zeros(1, S, dtype=torch.long, device="cuda")
    comp = rtkv.RealTimePrefillCompressor(cfg)
    comp.compress_layer_kv_cache(K, V, W, ids, 0)  # warm-up (first launches)
    comp.reset_compression_state()
    created = []
    orig = torch.cuda.Event

    def counting(*a, **k):  # (torch.cuda.Event constructs in __new__: wrap, do not subclass)
        e = orig(*a, **k)
        created.append(e)
        return e
    spans = []
    for l in range(layers):
        torch.cuda.synchronize()
        e0, e1 = orig(enable_timing=True), orig(enable_timing=True)
        e0.record()
        torch.cuda.Event = counting
        try:
            comp.compress_layer_kv_cache(K, V, W, ids, l)
        finally:
            torch.cuda.Event = orig
        e1.record()
        e1.synchronize()
        spans.append(e0.elapsed_time(e1) / 1e3)
    assert len(created) == layers, len(created)  # the completion event of each layer, nothing else
    times = [comp.layer_states[l]["device_processing_time"] for l in range(layers)]
    for t, span in zip(times, spans):
        assert 0.3 * span < t <= span * 1.02 + 2e-6, (t, span)


@pytest.mark.parametrize("strict", [True, False])
def test_processing_time_is_the_callers_wall_time(strict):
    """processing_time is the reference's quantity (unified_compressor.py:118,148): the wall time of each
    call as its caller sees it, so total_processing_time is LongBench's TTFT (longbench_eval.py:160, the
    sum over the layers).  Σ processing_time over 32 calls lies within the wall time of the 32 calls plus
    the final sync, and each layer's device span (device_processing_time) is positive."""
    import time
    import rtkv
    S, F, layers = 4096, 4096, 32
    cfg = rtkv.CompressionConfig(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25, num_hidden_layers=layers,
                                 high_precision_bits=8, medium_precision_bits=4, low_precision_bits=2)
    g = torch.Generator(device="cuda").manual_seed(11)
    P = rtkv.prompt_length(S)
    K = torch.randn(1, S, F, device="cuda", generator=g)
    V = torch.randn(1, S, F, device="cuda", generator=g)
    W = torch.rand(1, 32, S, P, device="cuda", generator=g)
    ids = torch.zeros(1, S, dtype=torch.long, device="cuda")
    comp = rtkv.RealTimePrefillCompressor(cfg, strict=strict)
    comp.compress_layer_kv_cache(K, V, W, ids, 0)  # warm-up
    comp.reset_compression_state()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for l in range(layers):
        comp.compress_layer_kv_cache(K, V, W, ids, l)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    total = comp.get_overall_compression_stats()["total_processing_time"]
    times = [comp.layer_states[l]["processing_time"] for l in range(layers)]
    assert total == pytest.approx(sum(times))
    assert 0.0 < total <= wall, (total, wall)
    # the calls are the whole loop but for the last layer's K4 tail: most of the wall time is inside them
    assert total >= 0.5 * wall, (total, wall)
    assert all(comp.layer_states[l]["device_processing_time"] > 0 for l in range(layers))


def test_device_span_does_not_depend_on_the_row_order():
    """The layer's device span (rtkv_layer_times: K1's first block to the K4 end stamp, the source of
    device_processing_time) against HIP events on the stream, on a layer whose 8-bit rows are the first kept
    rows and on one whose 8-bit rows are the last: only the waves of K4's last 2048 row tasks stamp the end
    (quant_impl.h kStampWindow), so if earlier, longer tasks finished after them the span would be short
    when the heavy rows come first.  Through the drop-in's own begin / finish calls: the begin
    call records the first event right before K1 (start_event), the second is recorded after K4 is enqueued,
    so only K1, K2, the host's reaction to the early statistics and K4 lie between them.  Measured on MI355X:
    events − stamps = 17.5 us in both orders (the events' own start / end latency,
    profiles/r06v_span_vs_events.log) — the stamps lose nothing to the row order."""
    import rtkv
    from rtkv import _lib as L
    from rtkv.engine import EarlyStatsBuffer, compress_layer_begin
    S, F = 16384, 4096
    cfg = rtkv.CompressionConfig(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25, num_hidden_layers=1,
                                 layer_weights=[1.0], high_precision_bits=8, medium_precision_bits=4,
                                 low_precision_bits=2)
    g = torch.Generator(device="cuda").manual_seed(21)
    P = rtkv.prompt_length(S)
    K = torch.randn(1, S, F, device="cuda", generator=g)
    V = torch.randn(1, S, F, device="cuda", generator=g)
    W0 = torch.rand(1, 32, S, P, device="cuda", generator=g)
    params = rtkv.params_from_config(cfg, 0, P, 0.6, L.EMIT_DEQUANT | L.EMIT_PACKED)
    ws = rtkv.Workspace("cuda")
    early = EarlyStatsBuffer()
    med = {}
    for order in ("high_first", "low_first"):
        ramp = torch.linspace(1.0, 0.01, S, device="cuda")  # early tokens most important
        if order == "low_first":
            ramp = ramp.flip(0)
        W = W0 * ramp.view(1, 1, S, 1)
        gaps = []
        for it in range(10):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            bufs = rtkv.LayerBuffers(1, S, F, K.dtype, "cuda", (2, 4, 8), outputs=False)
            e0.record()  # (creates the event and marks it recorded for torch; begin re-records it before K1)
            pend = compress_layer_begin(K, V, W, params, bufs, ws, early, start_event=e0.cuda_event)
            pend.stats()
            pend.finish()
            e1.record()
            torch.cuda.synchronize()
            ev, dev = e0.elapsed_time(e1) * 1e3, pend.device_seconds() * 1e6
            if it >= 2:  # (warm-up: the first calls' allocations)
                gaps.append((round(ev, 2), round(dev, 2)))
        print(f"device span vs events ({order}), us:", gaps)
        labels = bufs.labels[0].cpu().numpy()
        kept = bufs.kept_index[0].cpu().numpy()[: pend.stats().max_kept]
        hi = 0 if order == "high_first" else len(kept) - 64
        assert (labels[kept[hi:hi + 64]] == 2).all()  # the 8-bit (high-precision) rows are first / last
        for ev, dev in gaps:
            assert 0 < dev <= ev + 2.0, gaps  # the stamps lie inside the events
        med[order] = float(np.median([ev - dev for ev, dev in gaps]))
        assert med[order] <= 30.0, med
    assert abs(med["high_first"] - med["low_first"]) <= 4.0, med  # no order-dependent loss of K4's tail
