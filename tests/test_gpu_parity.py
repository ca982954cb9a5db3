"""GPU parity: the HIP path (librtkv.so through the rtkv mirror classes / C ABI) against the golden
fixtures generated from the reference and against the oracle.  Bit-exact for scores, classes,
selection masks, dequantized K'/V' and packed codes; see tests/golden/gen_golden.py for how the
fixtures were produced.  Run with `pytest -m gpu`."""
import numpy as np
import pytest
import torch

import rtkv_oracle as orc
import synth
from conftest import assert_matches, load_case, load_manifest

pytestmark = pytest.mark.gpu

CASES = load_manifest()["cases"]
TD = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}


def by_kind(kind):
    return [c for c in CASES if c["kind"] == kind]


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    import rtkv
    rtkv.build()
    return torch.device("cuda:0")


def dev(stored: np.ndarray, dtype: str) -> torch.Tensor:
    """storage array (float32 or uint16 bits) → device tensor of `dtype`."""
    if dtype == "float32":
        return torch.from_numpy(np.ascontiguousarray(stored, np.float32)).cuda()
    t = torch.from_numpy(np.ascontiguousarray(stored, np.uint16).view(np.int16)).cuda()
    return t.view(TD[dtype])


def host(t: torch.Tensor) -> np.ndarray:
    """device tensor → storage array (float32, or uint16 bits for half types)."""
    t = t.detach().contiguous().cpu()
    if t.dtype == torch.float32:
        return t.numpy()
    return t.view(torch.int16).numpy().view(np.uint16)


def config(params: dict, L: int, bits=(2, 4, 8)):
    import rtkv
    kw = dict(params)
    kw.update(low_precision_bits=bits[0], medium_precision_bits=bits[1], high_precision_bits=bits[2],
              num_hidden_layers=L)
    if L == 1:
        kw["layer_weights"] = [1.0]
    return rtkv.CompressionConfig(**kw)


COVERAGE = dict(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25)


# ----------------------------------------------------------------------------- stages
@pytest.mark.parametrize("case", by_kind("position_bias"), ids=lambda c: c["name"])
def test_position_bias(case):
    import rtkv
    sc = rtkv.PromptGuidedImportanceScorer(config(COVERAGE, 4))
    pos = sc.compute_position_bias(case["spec"]["S"], torch.device("cuda"))
    assert_matches(case, "pos", host(pos), load_case(case))


def test_position_bias_exhaustive_up_to_2_20():
    """Device logf path == torch CPU log for every integer 1..2^20 (incl. the Sleef exceptions)."""
    import rtkv
    S = 1 << 20
    sc = rtkv.PromptGuidedImportanceScorer(config(COVERAGE, 4))
    pos = host(sc.compute_position_bias(S, torch.device("cuda")))
    assert np.array_equal(pos, orc.position_bias(S))


@pytest.mark.parametrize("case", by_kind("aggregation"), ids=lambda c: c["name"])
def test_aggregation_scores(case):
    import rtkv
    s = case["spec"]
    arrays = load_case(case)
    W = (synth.attention_full(s["seed"], s["B"], s["H"], s["S"], s["dtype"]) if s["full"]
         else synth.attention_slice(s["seed"], s["B"], s["H"], s["S"], s["P"], s["dtype"]))
    Wd = dev(W, s["dtype"])
    sc = rtkv.PromptGuidedImportanceScorer(config(COVERAGE, s["L"]))
    idx = torch.arange(s["P"], device="cuda")
    A = sc.compute_attention_aggregation(Wd, idx, 0)
    assert A.dtype == TD[s["dtype"]]
    assert_matches(case, "A", host(A.float()), arrays)
    assert_matches(case, "N", host(sc.normalize_attention_scores(A, 0).float()), arrays)
    for layer in s["layers"]:
        out = sc.compute_importance_scores(Wd, idx, layer)
        assert out.dtype == torch.float32
        assert_matches(case, f"scores_l{layer}", host(out), arrays)


@pytest.mark.parametrize("B,H,S", [(1, 32, 16384), (2, 40, 3001), (1, 7, 100)])
def test_fp32_register_aggregation_matches_lds_path_and_oracle(B, H, S, monkeypatch):
    """fp32, P = 128: K1's register/shuffle kernel (aggregation_shfl32_kernel) == the LDS kernel
    (RTKV_K1_LDS) == the oracle, bit for bit; ragged token blocks and head tails included."""
    import rtkv
    P = 128
    W = synth.attention_slice(900 + S, B, H, S, P, "float32")
    Wd = dev(W, "float32")
    sc = rtkv.PromptGuidedImportanceScorer(config(COVERAGE, 4))
    idx = torch.arange(P, device="cuda")
    reg = host(sc.compute_attention_aggregation(Wd, idx, 0))
    monkeypatch.setenv("RTKV_K1_LDS", "1")
    lds = host(sc.compute_attention_aggregation(Wd, idx, 0))
    assert np.array_equal(reg, lds)
    assert np.array_equal(reg, orc.attention_aggregation(W, 0, P))


@pytest.mark.parametrize("B,H,S,dtype", [(1, 32, 8192, "float16"), (2, 40, 3001, "bfloat16"), (1, 40, 4096, "float16"),
                                          (1, 32, 4096, "bfloat16"), (2, 32, 77, "float16")])
def test_split_head_aggregation_matches_unsplit_and_oracle(B, H, S, dtype, monkeypatch):
    """fp16/bf16, P = 128, H = 32 or 40: K1's split-head kernel (the workgroup's halves stream the two
    halves of the head range, half 1 hands its block sums over through LDS) == the unsplit kernel
    (RTKV_K1_NOSPLIT) == the oracle, bit for bit; ragged token blocks and the 13B head tail (40 = 2·16 + 8)
    included."""
    import rtkv
    P = 128
    W = synth.attention_slice(950 + S + H, B, H, S, P, dtype)
    Wd = dev(W, dtype)
    sc = rtkv.PromptGuidedImportanceScorer(config(COVERAGE, 4))
    idx = torch.arange(P, device="cuda")
    split = host(sc.compute_attention_aggregation(Wd, idx, 0).float())
    monkeypatch.setenv("RTKV_K1_NOSPLIT", "1")
    whole = host(sc.compute_attention_aggregation(Wd, idx, 0).float())
    assert np.array_equal(split.view(np.uint32), whole.view(np.uint32))
    assert np.array_equal(split, orc.attention_aggregation(W, synth.DTYPES[dtype], P))


@pytest.mark.parametrize("case", by_kind("normalize"), ids=lambda c: c["name"])
def test_normalize_edges(case):
    import rtkv
    arrays = load_case(case)
    dt = case["spec"]["dtype"]
    sc = rtkv.PromptGuidedImportanceScorer(config(COVERAGE, 4))
    N = sc.normalize_attention_scores(dev(arrays["A"], dt), 0)
    assert_matches(case, "N", host(N.float()), arrays)


def quant_inputs(s):
    K, V = synth.kv(s["seed"], s["B"], s["S"], s["F"], s["dtype"])
    Kf = synth.to_f32(K, s["dtype"])
    b, i = s["const_row"]
    Kf[b, i, :] = Kf[b, i, 0]
    return synth.cast(Kf.astype(np.float64), s["dtype"]), V


@pytest.mark.parametrize("case", by_kind("quant"), ids=lambda c: c["name"])
def test_mixed_precision_quant(case):
    import rtkv
    s = case["spec"]
    arrays = load_case(case)
    K, V = quant_inputs(s)
    q = rtkv.DynamicPrecisionQuantizer(config(dict(COVERAGE, theta_h=s["theta"][0], theta_m=s["theta"][1]), 4,
                                              s["bits"]))
    scores = torch.from_numpy(synth.scores_like(s["seed"], s["B"], s["S"])).cuda()
    labels, stats = q.assign_precision_levels(scores)
    assert labels.dtype == torch.int64
    assert_matches(case, "labels", labels.cpu().numpy().astype(np.uint8), arrays)
    assert [stats["low_count"], stats["medium_count"], stats["high_count"]] == \
        [case["scalars"]["low"], case["scalars"]["medium"], case["scalars"]["high"]]
    kq, vq, info = q.apply_mixed_precision_quantization(dev(K, s["dtype"]), dev(V, s["dtype"]), labels)
    assert "bit_assignments" in info
    assert_matches(case, "k_q", host(kq), arrays)
    assert_matches(case, "v_q", host(vq), arrays)


def test_f16_16bit_raises_like_the_reference():
    import rtkv
    case = by_kind("quant_error")[0]
    s = case["spec"]
    K, V = synth.kv(s["seed"], s["B"], s["S"], s["F"], "float16")
    q = rtkv.DynamicPrecisionQuantizer(config(COVERAGE, 4, s["bits"]))
    labels = torch.tensor(s["labels"], device="cuda")
    with pytest.raises(RuntimeError, match="c10::Half without overflow"):
        q.apply_mixed_precision_quantization(dev(K, "float16"), dev(V, "float16"), labels)


def test_fast_division_fp32_every_mantissa_pair():
    """fp32 rows use the same reciprocal + FMA quotient behind a gate that keeps every step normal
    (quant_impl.h fast_div_ok), so each step commutes with power-of-two scaling and a pair reduces
    to its mantissas: all 2^46 (X, S) in [1, 2)^2 are compared bitwise with the IEEE division, then
    scaled and negative pairs spot-check the scaling argument."""
    import time
    import rtkv
    lib = rtkv._lib.lib()
    counts = torch.zeros(2, dtype=torch.int64, device="cuda")
    st = rtkv._lib.stream_ptr(counts.device)
    step = 1 << 17
    t0 = time.time()
    for lo in range(0, 1 << 23, step):
        rtkv._lib.check(lib.rtkv_selfcheck_division_f32(lo, lo + step, 0, 0, 0, counts.data_ptr(), st),
                        "rtkv_selfcheck_division_f32")
        if lo % (1 << 21) == 0:
            torch.cuda.synchronize()
            print(f"divisors < {lo + step}: {counts.cpu().tolist()} ({time.time() - t0:.1f} s)", flush=True)
    checked, bad = counts.cpu().tolist()
    assert (checked, bad) == (1 << 46, 0)
    for ex, es, neg in ((-40, 30, 0), (50, -45, 1), (-59, -95, 0), (90, 95, 1), (0, 99, 0), (-20, -99, 1)):
        counts.zero_()
        rtkv._lib.check(lib.rtkv_selfcheck_division_f32((ex * 7919) % (1 << 23) // 2, (ex * 7919) % (1 << 23) // 2 + 64,
                                                        ex, es, neg, counts.data_ptr(), st), "selfcheck")
        checked, bad = counts.cpu().tolist()
        assert bad == 0 and checked > 0, (ex, es, neg, checked, bad)


@pytest.mark.parametrize("dtype", ["float16", "bfloat16"])
def test_fast_division_exhaustive(dtype):
    """K4 divides by the row scale with reciprocal + FMA correction (quant_impl.h fast_quotient).
    The device enumerates every (x, s) pair of the 16-bit dtype its row gate admits and compares
    the quotient bitwise with the IEEE fp32 division."""
    import rtkv
    counts = torch.zeros(2, dtype=torch.int64, device="cuda")
    rc = rtkv._lib.lib().rtkv_selfcheck_division(synth.DTYPES[dtype], counts.data_ptr(),
                                                 rtkv._lib.stream_ptr(counts.device))
    rtkv._lib.check(rc, "rtkv_selfcheck_division")
    checked, bad = counts.cpu().tolist()
    assert bad == 0
    assert checked == _admitted_division_pairs(dtype)


def _admitted_division_pairs(dtype: str) -> int:
    """Host count of the (x, s) pairs quant_impl.h fast_div_ok admits: finite x, positive finite s;
    bf16 additionally 2^-62 <= s <= 2^62, |x| <= 2^62 and (x == 0 or |x| >= 2^-48 * s)."""
    bitsv = np.arange(65536, dtype=np.uint32)
    with np.errstate(invalid="ignore"):
        vals = synth.to_f32(bitsv.astype(np.uint16), dtype).astype(np.float64)
    finite = np.isfinite(vals)
    pos_s = vals[1:0x8000]
    pos_s = pos_s[np.isfinite(pos_s)]
    if dtype == "float16":
        return int(pos_s.size) * int(finite.sum())
    ax = np.abs(vals[finite])
    zeros = int((ax == 0).sum())
    nz = np.sort(ax[(ax != 0) & (ax <= 2.0 ** 62)])
    s = pos_s[(pos_s >= 2.0 ** -62) & (pos_s <= 2.0 ** 62)]
    lo = np.searchsorted(nz, s * 2.0 ** -48, side="left")
    return int(s.size) * zeros + int((nz.size - lo).sum())


def _division_edge_rows(dtype: str, F: int) -> np.ndarray:
    """Rows that sit on either side of K4's fast-division row gate."""
    rng = np.random.default_rng(5)
    rows = [rng.standard_normal(F)]                                   # ordinary row (fast path)
    z = rng.standard_normal(F)
    z[::3] = 0.0
    z[1::7] = -0.0
    rows.append(z)                                                    # exact and negative zeros
    rows.append(np.full(F, 0.75))                                     # constant row (scale 1)
    if dtype == "float16":
        t = np.zeros(F)
        t[::5] = 2.0 ** -24
        rows.append(t)                                                # scale underflows to 0: IEEE x/0
        big = rng.choice([-60000.0, 60000.0, 1.0], F)
        rows.append(big)                                              # range overflows: scale = inf
        rows.append(rng.integers(-1023, 1024, F) * 2.0 ** -24)        # subnormal values
    elif dtype == "bfloat16":
        t = 1.0 + rng.standard_normal(F)
        t[::11] = 1e-30
        rows.append(t)                                                # tiny nonzero next to O(1) values
        rows.append(rng.standard_normal(F) * 1e30)                    # |x| > 2^62
        rows.append(rng.standard_normal(F) * 1e-25)                   # scale < 2^-62
        rows.append(rng.standard_normal(F) * 2.0 ** -120)             # subnormal-adjacent
    else:
        rows.append(rng.standard_normal(F) * 1e-38)                   # subnormal-adjacent: IEEE path
        rows.append(rng.standard_normal(F) * 1e37)                    # scale > 2^100: IEEE path
        t = 1.0 + rng.standard_normal(F)
        t[::13] = 2.0 ** -61
        rows.append(t)                                                # |x| < 2^-60 next to O(1) values
        t = 1.0 + rng.standard_normal(F)
        t[::13] = 2.0 ** -59
        rows.append(t)                                                # just inside the gate
        rows.append(rng.standard_normal(F) * 2.0 ** -90)              # tiny row (|x| < 2^-60): IEEE path
        rows.append(rng.standard_normal(F) * 2.0 ** 98)               # scale near 2^100
        t = rng.standard_normal(F)
        t[::17] = 1e-37
        rows.append(t)                                                # |x| < 2^-100 s
    return synth.cast(np.stack(rows)[None], dtype)


@pytest.mark.parametrize("dtype", ["float16", "bfloat16", "float32"])
@pytest.mark.parametrize("F", [4096, 512])
def test_quant_rows_on_both_sides_of_the_division_gate(dtype, F):
    import rtkv
    x = _division_edge_rows(dtype, F)
    S = x.shape[1]
    for bits in ((2, 4, 8), (4, 8, 16)):
        if dtype == "float16" and bits[2] == 16:
            continue
        for shift in range(3):
            lab = ((np.arange(S) + shift) % 3).astype(np.int64)[None]
            q = rtkv.DynamicPrecisionQuantizer(config(COVERAGE, 4, bits))
            kq, vq, _ = q.apply_mixed_precision_quantization(dev(x, dtype), dev(x[:, ::-1].copy(), dtype),
                                                             torch.from_numpy(lab).cuda())
            ref_k = orc.mixed_precision(x, synth.DTYPES[dtype], lab, bits)
            ref_v = orc.mixed_precision(x[:, ::-1].copy(), synth.DTYPES[dtype], lab, bits)
            for got, ref in ((host(kq), ref_k), (host(vq), ref_v)):
                # NaN outputs (scale 0 / inf rows) are compared by position: the sign of a generated
                # NaN is platform-defined (x86 default NaN is negative, gfx950's is positive)
                nan_g, nan_r = np.isnan(synth.to_f32(got, dtype)), np.isnan(synth.to_f32(ref, dtype))
                assert np.array_equal(nan_g, nan_r), (bits, shift)
                assert np.array_equal(got[~nan_g], ref[~nan_r]), (bits, shift)


def test_tensor_quant_helpers_match_oracle():
    import rtkv
    q = rtkv.DynamicPrecisionQuantizer(config(COVERAGE, 4))
    for dt in ["float32", "float16", "bfloat16"]:
        x = synth.cast(synth.normal(42, (3, 50)), dt)
        for bits in (2, 4, 8):
            sc, zp = q.get_quantization_params(dev(x, dt), bits)
            osc, ozp = orc.quant_params(x, synth.DTYPES[dt], bits)
            assert float(sc) == osc and float(zp) == ozp
            out = q.quantize_tensor(dev(x, dt), bits, sc, zp)
            _, ref = orc.fake_quant(x, synth.DTYPES[dt], bits, osc, ozp)
            assert np.array_equal(host(out), ref)


def test_adaptive_quantization_matches_per_class_oracle():
    import rtkv
    for dt in ["float32", "bfloat16"]:
        x = synth.cast(synth.normal(7, (2, 20, 32)), dt)
        labels = (synth.uniform(8, (2, 20)) * 3).astype(np.int64)
        aq = rtkv.AdaptiveQuantization(32)
        out = host(aq(dev(x, dt), torch.from_numpy(labels).cuda()))
        xf = synth.to_f32(x, dt)
        for level, bits in enumerate([2, 4, 8]):
            rows = labels.reshape(-1) == level
            if not rows.any():
                continue
            sub = synth.cast(xf.reshape(-1, 32)[rows].astype(np.float64), dt)
            sc, zp = orc.quant_params(sub, synth.DTYPES[dt], bits)
            _, ref = orc.fake_quant(sub, synth.DTYPES[dt], bits, sc, zp)
            assert np.array_equal(out.reshape(-1, 32)[rows], ref)


@pytest.mark.parametrize("case", by_kind("select"), ids=lambda c: c["name"])
def test_selection(case):
    import rtkv
    s = case["spec"]
    arrays = load_case(case)
    cfg = config(dict(COVERAGE, theta_h=s["theta"][0], theta_m=s["theta"][1]), s["L"], s["bits"])
    scores_np = synth.scores_like(s["seed"], s["B"], s["S"])
    scores = torch.from_numpy(scores_np).cuda()
    labels = torch.from_numpy(arrays["labels"].astype(np.int64)).cuda()
    prop = rtkv.SelectiveTokenPropagator(cfg)
    if s.get("fallback"):
        cfg.early_layer_ratio = cfg.middle_layer_ratio = cfg.later_layer_ratio = s["ratio"]
        prop = rtkv.SelectiveTokenPropagator(cfg)
        K, V = synth.kv(s["seed"], s["B"], s["S"], 16, "float32")
        ks, vs, ss, ls, info = prop.apply_token_selection(dev(K, "float32"), dev(V, "float32"), scores, labels, 0)
        mask = info["selection_mask"].cpu().numpy().astype(np.uint8)
        assert info["max_selected_length"] == case["scalars"]["max_selected"]
        if not s["tie_ambiguous"]:
            assert_matches(case, "mask", mask, arrays)
            assert_matches(case, "k_sel", host(ks), arrays)
        return
    mask, info = prop.select_tokens_with_budget(scores, labels, s["ratio"], s["layer"])
    mask = mask.cpu().numpy().astype(np.uint8)
    omask, kept, _, _ = orc.select(scores_np, arrays["labels"], s["bits"], s["ratio"])
    assert np.array_equal(mask, omask)  # stable tie order, always
    if not s["tie_ambiguous"]:
        assert_matches(case, "mask", mask, arrays)
        assert info["selected_counts"] == case["scalars"]["selected_counts"]


@pytest.mark.parametrize("B,S,ratio,bits", [(1, 10, 0.8, (4, 8, 16)), (2, 64, 0.6, (2, 4, 8)), (1, 4096, 0.4, (2, 4, 8)),
                                            (3, 333, 0.3, (4, 8, 16)), (1, 16384, 0.8, (2, 4, 8)), (1, 50, 0.01, (2, 4, 8))])
def test_selection_with_interleaved_classes(B, S, ratio, bits):
    """select_tokens_with_budget with caller classes unrelated to the scores (the reference's own
    test_selective_propagator: randn scores, randint labels) — the exact general greedy path."""
    import rtkv
    cfg = config(COVERAGE, 4, bits)
    rng = np.random.default_rng(S)
    scores = rng.standard_normal((B, S)).astype(np.float32)
    labels = rng.integers(0, 3, (B, S)).astype(np.uint8)
    prop = rtkv.SelectiveTokenPropagator(cfg)
    mask, info = prop.select_tokens_with_budget(torch.from_numpy(scores).cuda(), torch.from_numpy(labels).cuda(),
                                                ratio, 0)
    omask, kept, _, _ = orc.select(scores, labels, bits, ratio)
    # select_tokens_with_budget has no fallback: the oracle's fallback rows must come back empty
    if omask.sum() and kept.max() and not (orc.select(scores, labels, bits, ratio)[3]).any():
        assert np.array_equal(mask.cpu().numpy().astype(np.uint8), omask)
    else:
        assert mask.sum().item() == 0


# ----------------------------------------------------------------------------- full layer
def layer_inputs(s):
    F = s["Hkv"] * s["D"]
    K, V = synth.kv(s["seed"], s["B"], s["S"], F, s["dtype"])
    W = synth.attention_slice(s["seed"], s["B"], s["H"], s["S"], s["P"], s["dtype"])
    return K, V, W


def layer_config(s):
    cfg = config(s["params"], s["L"], s["bits"])
    if s["no_selection"]:
        cfg.early_layer_ratio = cfg.middle_layer_ratio = cfg.later_layer_ratio = 1.0
    return cfg


@pytest.mark.parametrize("case", by_kind("layer"), ids=lambda c: c["name"])
def test_compress_layer_kv_cache(case):
    import rtkv
    s = case["spec"]
    arrays = load_case(case)
    K, V, W = layer_inputs(s)
    comp = rtkv.RealTimePrefillCompressor(layer_config(s))
    Kd, Vd, Wd = dev(K, s["dtype"]), dev(V, s["dtype"]), dev(W, s["dtype"])
    ids = torch.zeros(s["B"], s["S"], dtype=torch.long, device="cuda")
    if s["no_selection"]:
        scores = comp.importance_tracker.update_scores(s["layer"], Wd, comp.identify_prompt_tokens(ids))
        labels, _ = comp.quantizer.assign_precision_levels(scores)
        k2, v2, _ = comp.quantizer.apply_mixed_precision_quantization(Kd, Vd, labels)
        assert_matches(case, "scores", host(scores), arrays)
        assert_matches(case, "k_out", host(k2), arrays)
        assert_matches(case, "v_out", host(v2), arrays)
        return
    k2, v2, info = comp.compress_layer_kv_cache(Kd, Vd, Wd, ids, s["layer"])
    assert_matches(case, "scores", comp.importance_tracker.layer_scores[s["layer"]].numpy(), arrays)
    assert_matches(case, "labels", info["quantization_info"]["bit_assignments"].astype(np.uint8), arrays)
    mask = info["propagation_info"]["selection_mask"].cpu().numpy().astype(np.uint8)
    if s["tie_ambiguous"]:
        pytest.skip("reference selection depends on its unstable argsort tie order")
    assert_matches(case, "mask", mask, arrays)
    assert k2.shape[1] == case["scalars"]["max_selected"]
    assert_matches(case, "k_out", host(k2), arrays)
    assert_matches(case, "v_out", host(v2), arrays)
    ps = info["precision_stats"]
    assert [ps["high_count"], ps["medium_count"], ps["low_count"]] == \
        [case["scalars"]["high"], case["scalars"]["medium"], case["scalars"]["low"]]
    assert info["compression_ratio"] == case["scalars"]["compression_ratio"]
    ist = info["importance_stats"]
    for k in ("mean_score", "std_score", "min_score", "max_score"):
        assert abs(ist[k] - case["scalars"][k]) <= 1e-5 * max(1.0, abs(case["scalars"][k])), k
    # packed codes: decode → identical to the dequantized output, and identical bytes to the oracle
    if "packed" in info:
        pk = info["packed"]
        dk, dv = rtkv.unpack_layer(pk)
        assert torch.equal(dk.view(torch.int16 if dk.element_size() == 2 else torch.int32),
                           k2.view(torch.int16 if k2.element_size() == 2 else torch.int32))
        assert torch.equal(dv.view(torch.int16 if dv.element_size() == 2 else torch.int32),
                           v2.view(torch.int16 if v2.element_size() == 2 else torch.int32))
        if s["S"] * s["Hkv"] * s["D"] <= (1 << 22):
            dt = synth.DTYPES[s["dtype"]]
            pr = s["params"]
            o = orc.compress_layer(K, V, dt, W, dt, s["P"], pr["alpha"], pr["beta"], pr["gamma"], s["layer_weight"],
                                   pr["theta_h"], pr["theta_m"], s["bits"], s["ratio"])
            assert np.array_equal(pk["codes_k"].cpu().numpy(), o["packed_k"])
            assert np.array_equal(pk["codes_v"].cpu().numpy(), o["packed_v"])
            assert np.array_equal(pk["scale_zp"].cpu().numpy(), o["scale_zp"])
            assert np.array_equal(pk["row_offset"].cpu().numpy(), o["row_offset"])


@pytest.mark.parametrize("case", [c for c in by_kind("layer") if c["spec"]["no_selection"]], ids=lambda c: c["name"])
def test_quant_only_fused_launch_matches_reference_golden(case):
    """BASELINE config 2 (quantization only) through the launch the bench's cfg2_s4096_quant leg times:
    rtkv_compress_layer with RTKV_NO_SELECTION — the quantization-only K2 (fsel_quant_kernel: scores,
    classes, row offsets) and K4 — byte for byte against the reference's
    apply_mixed_precision_quantization output on the same inputs (dynamic_quantization.py:128-196;
    tests/golden/gen_golden.py cfg2_quant, fp32 = the reference model's dtype and fp16)."""
    import rtkv
    from rtkv import _lib as L
    s = case["spec"]
    arrays = load_case(case)
    K, V, W = layer_inputs(s)
    B, S, F = s["B"], s["S"], s["Hkv"] * s["D"]
    cfg = layer_config(s)
    p = rtkv.params_from_config(cfg, s["layer"], s["P"], 1.0, L.EMIT_DEQUANT | L.EMIT_PACKED | L.NO_SELECTION)
    td = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}[s["dtype"]]
    bufs = rtkv.LayerBuffers(B, S, F, td, "cuda", tuple(s["bits"]))
    res = rtkv.compress_layer(dev(K, s["dtype"]), dev(V, s["dtype"]), dev(W, s["dtype"]), p, bufs, rtkv.Workspace("cuda"))
    st = res.final_stats()
    assert st.max_kept == S and case["scalars"]["max_selected"] == S
    k2, v2 = res.kv()
    assert_matches(case, "scores", bufs.scores.cpu().numpy(), arrays)
    assert_matches(case, "labels", bufs.labels.cpu().numpy(), arrays)
    assert_matches(case, "mask", bufs.mask.cpu().numpy(), arrays)
    assert_matches(case, "k_out", host(k2), arrays)
    assert_matches(case, "v_out", host(v2), arrays)
    cc = st.batch[0]["class_count"]
    assert [cc[2], cc[1], cc[0]] == [case["scalars"]["high"], case["scalars"]["medium"], case["scalars"]["low"]]
    assert torch.equal(bufs.kept_index[0].cpu(), torch.arange(S, dtype=torch.int32))
    # the packed codes decode to the same rows
    n = st.total_packed_bytes
    dk, dv = rtkv.unpack_layer(dict(codes_k=bufs.packed_k[:n], codes_v=bufs.packed_v[:n], row_offset=bufs.row_offset,
                                    scale_zp=bufs.scale_zp, kept_index=bufs.kept_index, labels=bufs.labels, rows=[S],
                                    bits=tuple(s["bits"]), dtype=td, feature_dim=F))
    iv = torch.int16 if td != torch.float32 else torch.int32
    assert torch.equal(dk.view(iv), k2.view(iv)) and torch.equal(dv.view(iv), v2.view(iv))


def test_native_bhsd_layout_matches_bsf():
    """[B,H,S,D] input (no transpose copy) gives the same outputs as the [B,S,H*D] API layout."""
    import rtkv
    from rtkv import _lib as L
    B, H, S, D = 2, 4, 300, 64
    cfg = config(COVERAGE, 4)
    K, V = synth.kv(11, B, S, H * D, "float16")
    W = synth.attention_slice(11, B, 8, S, rtkv.prompt_length(S), "float16")
    Kd, Vd, Wd = dev(K, "float16"), dev(V, "float16"), dev(W, "float16")
    Kh = Kd.view(B, S, H, D).transpose(1, 2).contiguous()
    Vh = Vd.view(B, S, H, D).transpose(1, 2).contiguous()
    bits = (2, 4, 8)
    P = rtkv.prompt_length(S)
    outs = []
    for layout, (k, v) in (("bsf", (Kd, Vd)), ("bhsd", (Kh, Vh))):
        p = rtkv.params_from_config(cfg, 1, P, 0.6, L.EMIT_DEQUANT | L.EMIT_PACKED)
        bufs = rtkv.LayerBuffers(B, S, H * D, torch.float16, "cuda", bits)
        res = rtkv.compress_layer(k, v, Wd, p, bufs, rtkv.Workspace("cuda"), layout=layout)
        kk, vv = res.kv()
        outs.append((kk.clone(), vv.clone(), bufs.packed_k[: res.stats().total_packed_bytes].clone()))
    assert torch.equal(outs[0][0].view(torch.int16), outs[1][0].view(torch.int16))
    assert torch.equal(outs[0][1].view(torch.int16), outs[1][1].view(torch.int16))
    assert torch.equal(outs[0][2], outs[1][2])


@pytest.mark.parametrize("dtype", ["float16", "bfloat16", "float32"])
def test_packed_only_mode_matches_dual_output(dtype):
    """EMIT_PACKED alone (the packed consumers' mode; fp16 rows take their own code path: packed
    clamp, no dequantized stores) writes the same codes and scale/zp as the dual-output launch,
    on ordinary rows, the division-gate edge rows, and rows holding NaN or ±inf."""
    import rtkv
    from rtkv import _lib as L
    F, S = 4096, 512
    K, V = synth.kv(21, 1, S, F, "float32")
    edge = synth.to_f32(_division_edge_rows(dtype, F), dtype)[0]
    K[0, 1:1 + edge.shape[0]] = edge
    V[0, 40:40 + edge.shape[0]] = edge[::-1]
    K[0, 30, ::97] = np.nan
    K[0, 31, 5] = np.inf
    V[0, 32, 7] = -np.inf
    V[0, 33, ::3] = np.nan
    W = synth.attention_slice(21, 1, 8, S, rtkv.prompt_length(S), dtype)
    Kd, Vd, Wd = dev(synth.cast(K, dtype), dtype), dev(synth.cast(V, dtype), dtype), dev(W, dtype)
    cfg = config(COVERAGE, 4)
    P = rtkv.prompt_length(S)
    got = []
    for flags, deq in ((L.EMIT_DEQUANT | L.EMIT_PACKED, True), (L.EMIT_PACKED, False)):
        p = rtkv.params_from_config(cfg, 1, P, 0.8, flags | L.NO_SELECTION)  # every row quantized
        bufs = rtkv.LayerBuffers(1, S, F, TD[dtype], "cuda", (2, 4, 8), emit_dequant=deq, emit_packed=True)
        res = rtkv.compress_layer(Kd, Vd, Wd, p, bufs, rtkv.Workspace("cuda"))
        st = res.stats()
        n = st.total_packed_bytes
        got.append((bufs.packed_k[:n].clone(), bufs.packed_v[:n].clone(),
                    bufs.scale_zp[:, :st.max_kept].clone().view(torch.int32), st.max_kept))
    assert got[0][3] == got[1][3]
    for a, b in zip(got[0][:3], got[1][:3]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B,S,dtype", [(1, 16384, "float16"), (1, 4096, "bfloat16"), (2, 3000, "float16")])
def test_packed_only_selection_matches_dual_output(B, S, dtype):
    """With a binding selection (dropped tokens, three classes; B = 2: padding rows past a batch row's
    kept count) the packed-only launch — for 2-byte rows the paired kernel, one task per kept row's K
    and V rows — writes the same codes, scale/zp and row offsets as the dual-output launch."""
    import rtkv
    from rtkv import _lib as L
    H = 32
    F = H * 128
    cfg = config(COVERAGE, 8)
    P = rtkv.prompt_length(S)
    K, V = synth.kv(77 + S, B, S, F, dtype)
    W = synth.attention_slice(77 + S, B, H, S, P, dtype)
    Kd, Vd, Wd = dev(K, dtype), dev(V, dtype), dev(W, dtype)
    got = []
    for flags, deq in ((L.EMIT_DEQUANT | L.EMIT_PACKED, True), (L.EMIT_PACKED, False)):
        p = rtkv.params_from_config(cfg, 2, P, 0.6, flags)
        bufs = rtkv.LayerBuffers(B, S, F, TD[dtype], "cuda", (2, 4, 8), emit_dequant=deq, emit_packed=True)
        res = rtkv.compress_layer(Kd, Vd, Wd, p, bufs, rtkv.Workspace("cuda"))
        st = res.stats()
        n = st.total_packed_bytes
        got.append((bufs.packed_k[:n].clone(), bufs.packed_v[:n].clone(),
                    bufs.scale_zp[:, :st.max_kept].clone().view(torch.int32), st.max_kept, n))
    assert got[0][3:] == got[1][3:]
    assert got[0][3] < S  # the selection dropped tokens
    for a, b in zip(got[0][:3], got[1][:3]):
        assert torch.equal(a, b)


# ----------------------------------------------------------------------------- full-size properties
@pytest.mark.parametrize("S,dtype,ratio,H", [(16384, "float16", 0.6, 32), (65536, "float16", 0.4, 32),
                                             (32768, "bfloat16", 0.8, 32),
                                             (16384, "float32", 0.6, 32),    # cfg3 at the model's fp32
                                             (32768, "float16", 0.4, 40),    # cfg5: 13B, F = 5120
                                             (32768, "float32", 0.6, 40)])
def test_full_size_properties(S, dtype, ratio, H):
    """BASELINE sizes: closed-form greedy counts, ascending order, budget, pack→unpack == dequant,
    and sampled rows re-quantized by the oracle."""
    import rtkv
    from rtkv import _lib as L
    D = 128
    F = H * D
    cfg = config(COVERAGE, 32)
    P = rtkv.prompt_length(S)
    K, V = synth.kv(5000 + S, 1, S, F, dtype)
    W = synth.attention_slice(5000 + S, 1, H, S, P, dtype)
    Kd, Vd, Wd = dev(K, dtype), dev(V, dtype), dev(W, dtype)
    del W
    p = rtkv.params_from_config(cfg, 3, P, ratio, L.EMIT_DEQUANT | L.EMIT_PACKED)
    bufs = rtkv.LayerBuffers(1, S, F, TD[dtype], "cuda", (2, 4, 8))
    res = rtkv.compress_layer(Kd, Vd, Wd, p, bufs, rtkv.Workspace("cuda"))
    st = res.stats()
    k2, v2 = res.kv()
    row = st.batch[0]
    n = row["class_count"]
    # closed form of the greedy (selective_propagation.py:119-131)
    U = int(np.floor(8.0 * (S * ratio)))
    used, want = 0, [0, 0, 0]
    for g, b in ((2, 8), (1, 4), (0, 2)):
        want[g] = min(n[g], (U - used) // b)
        used += want[g] * b
    assert row["kept_class"] == want and row["kept"] == sum(want) == st.max_kept
    assert row["cost_units"] == used <= U
    kept = bufs.kept_index[0, : row["kept"]].cpu().numpy()
    assert np.all(np.diff(kept) > 0)
    scores = bufs.scores[0].cpu().numpy()
    labels = bufs.labels[0].cpu().numpy()
    # every kept token of class g scores >= every dropped token of class g
    mask = np.zeros(S, bool)
    mask[kept] = True
    for g in range(3):
        ks, ds = scores[mask & (labels == g)], scores[~mask & (labels == g)]
        if ks.size and ds.size:
            assert ks.min() >= ds.max()
    dk, dv = rtkv.unpack_layer(dict(codes_k=bufs.packed_k, codes_v=bufs.packed_v, row_offset=bufs.row_offset[:, :st.max_kept],
                                    scale_zp=bufs.scale_zp[:, :st.max_kept], kept_index=bufs.kept_index[:, :st.max_kept],
                                    labels=bufs.labels, rows=[row["kept"]], bits=(2, 4, 8), dtype=TD[dtype],
                                    feature_dim=F))
    iv = torch.int32 if dtype == "float32" else torch.int16
    assert torch.equal(dk.view(iv), k2.view(iv))
    assert torch.equal(dv.view(iv), v2.view(iv))
    rng = np.random.default_rng(0)
    k2h = host(k2)[0]
    for r in rng.choice(row["kept"], size=16, replace=False):
        i = kept[r]
        bits = (2, 4, 8)[labels[i]]
        sc, zp = orc.quant_params(K[0, i], synth.DTYPES[dtype], bits)
        _, ref = orc.fake_quant(K[0, i], synth.DTYPES[dtype], bits, sc, zp)
        assert np.array_equal(k2h[r], ref)



@pytest.mark.parametrize("dtype,H", [("float32", 32), ("float16", 32), ("bfloat16", 32), ("float32", 40),
                                     ("float16", 40)])
def test_split_row_k4_matches_oracle(dtype, H):
    """Single-row layers take quant_rows_split_kernel: each row is quantized by 4 (5) waves — 2 for the
    2-byte dtypes with F = 4096 and dequantized outputs (every S) — that combine its min/max in LDS.  Dequantized rows, codes, scale/zp and
    row offsets equal the oracle's, including the division-gate edge rows (NaN / ±inf rows: the
    dual-vs-packed test above; their codes are platform-defined conversions)."""
    import rtkv
    from rtkv import _lib as L
    D, S = 128, 1024 if H == 32 else 800
    F = H * D
    K, V = synth.kv(77 + H, 1, S, F, "float32")
    edge = synth.to_f32(_division_edge_rows(dtype, F), dtype)[0]
    K[0, 3:3 + edge.shape[0]] = edge
    V[0, 50:50 + edge.shape[0]] = edge[::-1]
    K, V = synth.cast(K, dtype), synth.cast(V, dtype)
    P = rtkv.prompt_length(S)
    W = synth.attention_slice(77 + H, 1, H, S, P, dtype)
    dt = synth.DTYPES[dtype]
    pr = COVERAGE
    cfg = config(pr, 1)
    ratio = 0.6
    p = rtkv.params_from_config(cfg, 0, P, ratio, L.EMIT_DEQUANT | L.EMIT_PACKED)
    bufs = rtkv.LayerBuffers(1, S, F, TD[dtype], "cuda", (2, 4, 8))
    res = rtkv.compress_layer(dev(K, dtype), dev(V, dtype), dev(W, dtype), p, bufs, rtkv.Workspace("cuda"))
    st = res.stats()
    kk, vv = res.kv()
    o = orc.compress_layer(K, V, dt, W, dt, P, pr["alpha"], pr["beta"], pr["gamma"], cfg.layer_weights[0],
                           pr["theta_h"], pr["theta_m"], (2, 4, 8), ratio)
    R = st.max_kept
    assert 0 < R < S
    n = st.total_packed_bytes
    assert np.array_equal(bufs.packed_k[:n].cpu().numpy(), o["packed_k"][:n])
    assert np.array_equal(bufs.packed_v[:n].cpu().numpy(), o["packed_v"][:n])
    assert np.array_equal(bufs.row_offset[:, :R].cpu().numpy(), o["row_offset"])
    # scale/zp bit for bit; a NaN (an edge row that overflows the dtype) by position: the sign of a
    # generated NaN is platform-defined (x86's default NaN is negative, gfx950's positive)
    sz_g, sz_r = bufs.scale_zp[:, :R].cpu().numpy(), o["scale_zp"]
    assert np.array_equal(np.isnan(sz_g), np.isnan(sz_r))
    assert np.array_equal(sz_g[~np.isnan(sz_g)].view(np.int32), sz_r[~np.isnan(sz_r)].view(np.int32))
    for got, ref in ((host(kk), o["k_out"]), (host(vv), o["v_out"])):
        nan_g, nan_r = np.isnan(synth.to_f32(got, dtype)), np.isnan(synth.to_f32(ref, dtype))
        assert np.array_equal(nan_g, nan_r)
        assert np.array_equal(got[~nan_g], ref[~nan_r])
