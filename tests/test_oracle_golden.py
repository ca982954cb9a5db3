"""CPU: the oracle (oracle/rtkv_oracle.c) reproduces every golden fixture generated from the
reference (tests/golden/gen_golden.py).  This pins the oracle; the GPU tests then compare the HIP
path against the same fixtures and against the oracle."""
import numpy as np
import pytest

import rtkv_oracle as orc
import synth
from conftest import assert_matches, load_case, load_manifest

CASES = load_manifest()["cases"]
BIG = 1 << 24  # elements; larger layer fixtures are covered by the GPU tests


def by_kind(kind):
    return [c for c in CASES if c["kind"] == kind]


@pytest.mark.parametrize("case", by_kind("position_bias"), ids=lambda c: c["name"])
def test_position_bias(case):
    arrays = load_case(case)
    assert_matches(case, "pos", orc.position_bias(case["spec"]["S"]), arrays)


@pytest.mark.parametrize("case", by_kind("aggregation"), ids=lambda c: c["name"])
def test_aggregation_and_scores(case):
    s = case["spec"]
    arrays = load_case(case)
    W = (synth.attention_full(s["seed"], s["B"], s["H"], s["S"], s["dtype"]) if s["full"]
         else synth.attention_slice(s["seed"], s["B"], s["H"], s["S"], s["P"], s["dtype"]))
    dt = synth.DTYPES[s["dtype"]]
    A = orc.attention_aggregation(W, dt, s["P"])
    assert_matches(case, "A", A, arrays)
    assert_matches(case, "N", orc.minmax_normalize(A, dt), arrays)
    from base_config_shim import coverage_config
    cfg = coverage_config(s["L"])
    for layer in s["layers"]:
        sc = orc.importance_scores(A, dt, s["P"], cfg["alpha"], cfg["beta"], cfg["gamma"], cfg["layer_weights"][layer])
        assert_matches(case, f"scores_l{layer}", sc, arrays)


@pytest.mark.parametrize("case", by_kind("normalize"), ids=lambda c: c["name"])
def test_normalize_edges(case):
    arrays = load_case(case)
    dt = case["spec"]["dtype"]
    A = synth.to_f32(arrays["A"], dt)
    assert_matches(case, "N", orc.minmax_normalize(A, synth.DTYPES[dt]), arrays)


def quant_inputs(s):
    K, V = synth.kv(s["seed"], s["B"], s["S"], s["F"], s["dtype"])
    Kf = synth.to_f32(K, s["dtype"])
    b, i = s["const_row"]
    Kf[b, i, :] = Kf[b, i, 0]
    K = synth.cast(Kf.astype(np.float64), s["dtype"])
    return K, V


@pytest.mark.parametrize("case", by_kind("quant"), ids=lambda c: c["name"])
def test_mixed_precision_quant(case):
    s = case["spec"]
    arrays = load_case(case)
    K, V = quant_inputs(s)
    scores = synth.scores_like(s["seed"], s["B"], s["S"])
    labels, counts = orc.assign_precision(scores, *s["theta"])
    assert_matches(case, "labels", labels, arrays)
    assert counts.tolist() == [case["scalars"]["low"], case["scalars"]["medium"], case["scalars"]["high"]]
    dt = synth.DTYPES[s["dtype"]]
    assert_matches(case, "k_q", orc.mixed_precision(K, dt, labels, s["bits"]), arrays)
    assert_matches(case, "v_q", orc.mixed_precision(V, dt, labels, s["bits"]), arrays)


def test_f16_16bit_is_an_error_in_the_reference():
    case = [c for c in CASES if c["kind"] == "quant_error"][0]
    assert "cannot be converted to type c10::Half without overflow" in case["scalars"]["error"]
    assert orc.field_width(1, 16) == 0


@pytest.mark.parametrize("case", by_kind("select"), ids=lambda c: c["name"])
def test_selection(case):
    s = case["spec"]
    arrays = load_case(case)
    scores = synth.scores_like(s["seed"], s["B"], s["S"])
    labels, _ = orc.assign_precision(scores, *s["theta"])
    assert_matches(case, "labels", labels, arrays)
    mask, kept, units, fb = orc.select(scores, labels, s["bits"], s["ratio"])
    if s.get("tie_ambiguous"):
        pytest.skip("reference selection depends on its unstable argsort tie order")
    assert_matches(case, "mask", mask, arrays)


@pytest.mark.parametrize("case", [c for c in by_kind("layer")
                                  if c["spec"]["S"] * c["spec"]["Hkv"] * c["spec"]["D"] <= BIG],
                         ids=lambda c: c["name"])
def test_full_layer(case):
    s = case["spec"]
    arrays = load_case(case)
    F = s["Hkv"] * s["D"]
    K, V = synth.kv(s["seed"], s["B"], s["S"], F, s["dtype"])
    W = synth.attention_slice(s["seed"], s["B"], s["H"], s["S"], s["P"], s["dtype"])
    dt = synth.DTYPES[s["dtype"]]
    pr = s["params"]
    o = orc.compress_layer(K, V, dt, W, dt, s["P"], pr["alpha"], pr["beta"], pr["gamma"], s["layer_weight"],
                           pr["theta_h"], pr["theta_m"], s["bits"], s["ratio"], no_selection=s["no_selection"],
                           threads=4)  # OpenMP oracle: same bytes at any thread count
    assert_matches(case, "scores", o["scores"], arrays)
    assert_matches(case, "labels", o["labels"], arrays)
    if s["tie_ambiguous"]:
        pytest.skip("reference selection depends on its unstable argsort tie order")
    assert_matches(case, "mask", o["mask"], arrays)
    assert o["max_kept"] == case["scalars"]["max_selected"]
    assert_matches(case, "k_out", o["k_out"], arrays)
    assert_matches(case, "v_out", o["v_out"], arrays)
    # packed codes decode to the same dequantized rows (oracle-side pack/unpack round trip)
    n = o["kept"][0]
    if n:
        w = orc.field_width(dt, s["bits"][o["labels"][0, o["kept_index"][0, 0]]])
        codes = orc.unpack_codes(o["packed_k"][o["row_offset"][0, 0]:], F, w)
        sc, zp = o["scale_zp"][0, 0, 0], o["scale_zp"][0, 0, 1]
        kf = synth.to_f32(K, s["dtype"])[0, o["kept_index"][0, 0]]
        codes2, _ = orc.fake_quant(synth.cast(kf.astype(np.float64), s["dtype"]), dt,
                                   s["bits"][o["labels"][0, o["kept_index"][0, 0]]], sc, zp)
        assert np.array_equal(codes, codes2)
