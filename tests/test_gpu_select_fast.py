"""GPU: the one-launch selection (select_fast.hip, taken for B = 1 and S <= 65536) against the
multi-workgroup pipeline (select.hip, forced with RTKV_SELECT_PIPELINE) and against the oracle.

Both paths must agree byte for byte on scores, classes, mask, kept indices, row offsets, packed
codes, scale/zero-point and the dequantized rows, and exactly on every integer statistic; the
double sums (score_sum, score_m2, kept_score_sum) agree to 1e-12 relative (different summation
trees).  Cases cover the row-length edges of the 1024-token workgroups (S = 1, 2, 17,
4097, 16383..16385, 32768, 40000, 65536), the emergency fallback, quantization-only, heavy score ties (β = 0
and a 3-valued attention mass) and all three dtypes."""
import numpy as np
import pytest
import torch

import rtkv_oracle as orc
import synth

pytestmark = pytest.mark.gpu

TD = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    import rtkv
    rtkv.build()


def dev(stored: np.ndarray, dtype: str) -> torch.Tensor:
    if dtype == "float32":
        return torch.from_numpy(np.ascontiguousarray(stored, np.float32)).cuda()
    return torch.from_numpy(np.ascontiguousarray(stored, np.uint16).view(np.int16)).cuda().view(TD[dtype])


def tied_attention(seed, H, S, P, dtype, levels=3):
    """A prompt slice whose head-mean prompt mass takes only `levels` distinct values."""
    u = synth.uniform(seed, (S,))
    lvl = np.floor(u * levels) / max(1, levels - 1)
    W = np.zeros((1, H, S, P), np.float32)
    W[0, :, :, 0] = lvl[None, :].astype(np.float32) * 0.5
    return synth.cast(W, dtype)


def run(K, V, W, dtype, S, F, cfg_kw, layer, ratio, flags):
    import rtkv
    from rtkv import _lib as L
    cfg = rtkv.CompressionConfig(num_hidden_layers=4, **cfg_kw)
    P = rtkv.prompt_length(S)
    bits = (cfg.low_precision_bits, cfg.medium_precision_bits, cfg.high_precision_bits)
    p = rtkv.params_from_config(cfg, layer, P, ratio, flags)
    bufs = rtkv.LayerBuffers(1, S, F, TD[dtype], "cuda", bits)
    res = rtkv.compress_layer(K, V, W, p, bufs, rtkv.Workspace("cuda"))
    st = res.stats()
    n = st.max_kept
    pb = st.total_packed_bytes
    out = dict(scores=bufs.scores.cpu(), labels=bufs.labels.cpu(), mask=bufs.mask.cpu(),
               kept=bufs.kept_index[0, :n].cpu(), row_offset=bufs.row_offset[0, :n].cpu(),
               scale_zp=bufs.scale_zp[0, :n].cpu(), pk=bufs.packed_k[:pb].cpu(), pv=bufs.packed_v[:pb].cpu(),
               k_out=bufs.k_out[: n * F].cpu(), v_out=bufs.v_out[: n * F].cpu())
    return out, st


COV = dict(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25, low_precision_bits=2, medium_precision_bits=4,
           high_precision_bits=8)
CASES = [
    # S, dtype, ratio, cfg overrides, attention kind
    (1, "float16", 0.8, {}, "rand"),
    (2, "float32", 0.6, {}, "rand"),
    (17, "bfloat16", 0.4, {}, "rand"),
    (512, "float16", 0.6, {}, "rand"),
    (4097, "float16", 0.4, {}, "rand"),
    (4096, "float32", 0.6, dict(low_precision_bits=4, medium_precision_bits=8, high_precision_bits=16), "rand"),
    (16383, "bfloat16", 0.8, {}, "rand"),
    (16384, "float16", 0.6, {}, "rand"),
    (16385, "float16", 0.4, {}, "rand"),
    (20000, "bfloat16", 0.6, {}, "rand"),
    (32768, "float16", 0.8, {}, "rand"),
    (3000, "float16", 0.0004, {}, "rand"),        # budget below one 8-bit row: emergency fallback
    (333, "float32", 0.001, {}, "rand"),          # fallback, k = int(0.1 S)
    (4096, "float16", 0.5, dict(beta=0.0), "tie"),     # 3 distinct scores: threshold inside a tie block
    (9000, "bfloat16", 0.3, dict(beta=0.0, gamma=0.0), "tie"),
    (5000, "float16", 0.5, dict(beta=0.0), "const"),   # every score equal (den <= eps): pure index order
    # heavy ties in the 32-tokens-per-thread rescan (16384 < S <= 32768): the tie cutoff index
    (24576, "float32", 0.4, dict(beta=0.0), "tie"),
    (32768, "bfloat16", 0.6, dict(beta=0.0), "const"),
    # 64 tokens per thread (32768 < S <= 65536: 33..64 workgroups; the north star's S = 64k and the sharded
    # prefill's replicated global selection), incl. heavy ties and class counts of exactly 65536
    (40000, "float16", 0.6, {}, "rand"),
    (65536, "float32", 0.6, {}, "rand"),
    (65535, "bfloat16", 0.4, {}, "rand"),
    (49153, "float16", 0.4, dict(beta=0.0), "tie"),
    (65536, "bfloat16", 0.6, dict(beta=0.0), "const"),
    (65536, "float16", 0.0002, {}, "rand"),      # emergency fallback over 65536 tokens
]


@pytest.mark.parametrize("S,dtype,ratio,over,kind", CASES, ids=lambda v: str(v))
def test_single_matches_pipeline_and_oracle(S, dtype, ratio, over, kind):
    import rtkv
    from rtkv import _lib as L
    H, D = 2, 64
    F = H * D
    P = rtkv.prompt_length(S)
    K, V = synth.kv(700 + S, 1, S, F, dtype)
    if kind == "rand":
        W = synth.attention_slice(700 + S, 1, H, S, P, dtype)
    elif kind == "tie":
        W = tied_attention(700 + S, H, S, P, dtype)
    else:
        W = synth.cast(np.full((1, H, S, P), 0.25, np.float32), dtype)
    Kd, Vd, Wd = dev(K, dtype), dev(V, dtype), dev(W, dtype)
    kw = dict(COV, **over)
    base = L.EMIT_DEQUANT | L.EMIT_PACKED
    a, sa = run(Kd, Vd, Wd, dtype, S, F, kw, 1, ratio, base)
    b, sb = run(Kd, Vd, Wd, dtype, S, F, kw, 1, ratio, base | L.SELECT_PIPELINE)
    for name in a:
        assert torch.equal(a[name].view(torch.uint8) if a[name].dtype != torch.uint8 else a[name],
                           b[name].view(torch.uint8) if b[name].dtype != torch.uint8 else b[name]), name
    assert (sa.max_kept, sa.total_packed_bytes, sa.error_flags, sa.score_min, sa.score_max) == \
        (sb.max_kept, sb.total_packed_bytes, sb.error_flags, sb.score_min, sb.score_max)
    ra, rb = sa.batch[0], sb.batch[0]
    for k in ("class_count", "kept", "kept_class", "cost_units", "packed_bytes", "fallback"):
        assert ra[k] == rb[k], k
    for x, y in ((sa.score_sum, sb.score_sum), (sa.score_m2, sb.score_m2), (ra["kept_score_sum"], rb["kept_score_sum"])):
        assert abs(x - y) <= 1e-12 * max(1.0, abs(y))
    if kind != "rand" or S <= 4097:
        cfg = rtkv.CompressionConfig(num_hidden_layers=4, **kw)
        dt = synth.DTYPES[dtype]
        bits = (cfg.low_precision_bits, cfg.medium_precision_bits, cfg.high_precision_bits)
        o = orc.compress_layer(K, V, dt, W, dt, P, kw["alpha"], kw["beta"], kw["gamma"], cfg.layer_weights[1],
                               kw["theta_h"], kw["theta_m"], bits, ratio)
        assert o["max_kept"] == sa.max_kept
        assert np.array_equal(a["mask"].numpy(), o["mask"])
        assert np.array_equal(a["kept"].numpy(), o["kept_index"][0])
        assert np.array_equal(a["row_offset"].numpy(), o["row_offset"][0])
        assert np.array_equal(a["pk"].numpy(), o["packed_k"])
        assert np.array_equal(a["pv"].numpy(), o["packed_v"])


@pytest.mark.parametrize("S,dtype,over", [(8192, "float16", {}), (1, "float32", {}), (17, "bfloat16", {}),
                                          (1024, "float16", {}), (1025, "float32", {}), (4096, "float32", {}),
                                          (16385, "bfloat16", {}), (32768, "float16", {}),
                                          (65536, "float32", {}), (50001, "float16", {}),
                                          (4096, "float32", dict(low_precision_bits=4, medium_precision_bits=8,
                                                                 high_precision_bits=16)),
                                          (5000, "float16", dict(beta=0.0))])
def test_no_selection_single_matches_pipeline(S, dtype, over):
    """Quantization only (RTKV_NO_SELECTION, BASELINE config 2): the one-pass K2 (fsel_quant_kernel: scores,
    classes, row offsets from the predecessors' class counts) against the pipeline and the oracle."""
    import rtkv
    from rtkv import _lib as L
    H, D = 4, 64
    F = H * D
    P = rtkv.prompt_length(S)
    K, V = synth.kv(91 + S, 1, S, F, dtype)
    W = synth.attention_slice(91 + S, 1, H, S, P, dtype)
    Kd, Vd, Wd = dev(K, dtype), dev(V, dtype), dev(W, dtype)
    kw = dict(COV, **over)
    base = L.EMIT_DEQUANT | L.EMIT_PACKED | L.NO_SELECTION
    a, sa = run(Kd, Vd, Wd, dtype, S, F, kw, 0, 0.5, base)
    b, sb = run(Kd, Vd, Wd, dtype, S, F, kw, 0, 0.5, base | L.SELECT_PIPELINE)
    assert sa.max_kept == S == sb.max_kept
    for name in a:
        assert torch.equal(a[name].view(torch.uint8) if a[name].dtype != torch.uint8 else a[name],
                           b[name].view(torch.uint8) if b[name].dtype != torch.uint8 else b[name]), name
    assert (sa.total_packed_bytes, sa.error_flags, sa.score_min, sa.score_max) == \
        (sb.total_packed_bytes, sb.error_flags, sb.score_min, sb.score_max)
    ra, rb = sa.batch[0], sb.batch[0]
    for k in ("class_count", "kept", "kept_class", "cost_units", "packed_bytes", "fallback"):
        assert ra[k] == rb[k], k
    for x, y in ((sa.score_sum, sb.score_sum), (sa.score_m2, sb.score_m2), (ra["kept_score_sum"], rb["kept_score_sum"])):
        assert abs(x - y) <= 1e-12 * max(1.0, abs(y))
    cfg = rtkv.CompressionConfig(num_hidden_layers=4, **kw)
    dt = synth.DTYPES[dtype]
    bits = (cfg.low_precision_bits, cfg.medium_precision_bits, cfg.high_precision_bits)
    o = orc.compress_layer(K, V, dt, W, dt, P, kw["alpha"], kw["beta"], kw["gamma"], cfg.layer_weights[0],
                           kw["theta_h"], kw["theta_m"], bits, 1.0, no_selection=True)
    assert o["max_kept"] == S
    assert np.array_equal(a["scores"].numpy(), o["scores"]) and np.array_equal(a["labels"].numpy(), o["labels"])
    assert np.array_equal(a["row_offset"].numpy(), o["row_offset"][0])
    assert np.array_equal(a["pk"].numpy(), o["packed_k"]) and np.array_equal(a["pv"].numpy(), o["packed_v"])


@pytest.mark.parametrize("B,S,ratio,monotone", [(2, 3000, 0.5, False), (1, 12000, 0.3, True),
                                                (3, 777, 0.0002, False), (1, 40000, 0.3, True)])
def test_pipeline_with_adversarial_caller_inputs(B, S, ratio, monotone):
    """Regression for the pipeline's digit search (select.hip find_digit: out-of-range LDS index when a
    histogram held fewer tokens than the quota, fixed in e2ffcc3): caller scores with ±inf, NaN and
    ties, caller labels outside {0, 1, 2} (treated as LOW), budgets from zero to above S, B > 1 and
    S > 32768.  The selection must finish and stay self-consistent: ascending unique in-range kept
    indices that match the mask and the statistics, and the top-10% fallback when nothing fits."""
    import rtkv
    rng = np.random.default_rng(S)
    scores = rng.standard_normal((B, S)).astype(np.float32)
    scores[:, ::97] = np.inf
    scores[:, 5::89] = -np.inf
    scores[:, 13::7] = 0.5  # a tie block
    if monotone:  # classes monotone in the score
        labels = np.where(scores >= 0.4, 2, np.where(scores >= 0.25, 1, 0)).astype(np.int64)
    else:
        scores[:, 11::83] = np.nan
        labels = rng.integers(0, 6, (B, S)).astype(np.int64)
    prop = rtkv.SelectiveTokenPropagator(rtkv.CompressionConfig(num_hidden_layers=4))
    sd, ld = torch.from_numpy(scores).cuda(), torch.from_numpy(labels).cuda()
    if S > 16384:  # caller classes go through the exact general path, limited to S <= 16384 (it says so)
        with pytest.raises(RuntimeError, match="S <= 16384"):
            prop.select_tokens_with_budget(sd, ld, ratio, 1)
        return
    mask, info = prop.select_tokens_with_budget(sd, ld, ratio, 1)
    K = torch.zeros(B, S, 8, device="cuda")
    ks, vs, ss, ls, pinfo = prop.apply_token_selection(K, K, sd, ld, 1)
    torch.cuda.synchronize()
    m = mask.cpu().numpy()
    pm = pinfo["selection_mask"].cpu().numpy()
    for b in range(B):
        kept = np.nonzero(pm[b])[0]
        assert kept.size >= 1  # fallback keeps the top max(1, int(0.1 S)) when nothing fits
        assert kept.size <= pinfo["max_selected_length"]
        assert np.all(np.diff(kept) > 0) and kept[-1] < S
    assert m.shape == (B, S) and m.dtype == bool
    assert ks.shape[1] == pinfo["max_selected_length"]

