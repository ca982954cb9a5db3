"""Multi-layer state parity: get_overall_compression_stats (unified_compressor.py:174-230),
get_cumulative_scores (token_importance.py:202-214) and reset_compression_state (:232-235) of the
rtkv mirror after a sequence of layers, against the same calls on the reference
(tests/golden/gen_golden.py gen_stats).  The two wall-clock sums are only checked for presence:
they time the machine, not the algorithm."""
import numpy as np
import pytest
import torch

import synth
from conftest import assert_matches, load_case, load_manifest

pytestmark = pytest.mark.gpu

CASES = [c for c in load_manifest()["cases"] if c["kind"] == "stats"]
TD = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}
TIMING_KEYS = ("total_processing_time", "avg_processing_time_per_layer")


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")


def dev(stored, dtype):
    if dtype == "float32":
        return torch.from_numpy(np.ascontiguousarray(stored, np.float32)).cuda()
    return torch.from_numpy(np.ascontiguousarray(stored, np.uint16).view(np.int16)).cuda().view(TD[dtype])


def run_sequence(s):
    import rtkv
    kw = dict(s["params"])
    kw.update(num_hidden_layers=s["L"], low_precision_bits=s["bits"][0], medium_precision_bits=s["bits"][1],
              high_precision_bits=s["bits"][2])
    comp = rtkv.RealTimePrefillCompressor(rtkv.CompressionConfig(**kw))
    F = s["Hkv"] * s["D"]
    ids = torch.zeros(s["B"], s["S"], dtype=torch.long, device="cuda")
    infos = []
    for k, layer in enumerate(s["layers"]):
        K, V = synth.kv(s["seed"] * 100 + k, s["B"], s["S"], F, s["dtype"])
        W = synth.attention_slice(s["seed"] * 100 + k, s["B"], s["H"], s["S"], s["P"], s["dtype"])
        _, _, info = comp.compress_layer_kv_cache(dev(K, s["dtype"]), dev(V, s["dtype"]), dev(W, s["dtype"]), ids, layer)
        infos.append(info)
    return comp, infos


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"])
def test_overall_stats_cumulative_scores_and_reset(case):
    s = case["spec"]
    exp = case["scalars"]
    arrays = load_case(case)
    comp, infos = run_sequence(s)
    for info, ref in zip(infos, exp["per_layer"]):
        assert info["layer_idx"] == ref["layer"]
        assert info["compressed_shape"][1] == ref["compressed_len"]
        assert info["compression_ratio"] == ref["compression_ratio"]
    overall = comp.get_overall_compression_stats()
    assert set(overall) == set(exp["overall"])
    for k in TIMING_KEYS:
        assert overall[k] > 0.0
    for k, v in exp["overall"].items():
        if k not in TIMING_KEYS:
            assert overall[k] == v, k
    assert overall["avg_processing_time_per_layer"] == overall["total_processing_time"] / len(s["layers"])
    special = {l: what for l, what in exp["cumulative_special"]}
    for l in s["queried"]:
        if l in special:
            if special[l] == "KeyError":
                with pytest.raises(KeyError):
                    comp.importance_tracker.get_cumulative_scores(l)
            else:
                assert comp.importance_tracker.get_cumulative_scores(l) is None
            continue
        c = comp.importance_tracker.get_cumulative_scores(l)
        assert c.device.type == "cpu" and c.dtype == torch.float32
        assert_matches(case, f"cum_l{l}", c.numpy(), arrays)
    comp.reset_compression_state()
    after = exp["after_reset"]
    assert comp.get_overall_compression_stats() == after["overall"] == {}
    assert comp.importance_tracker.get_cumulative_scores(0) is None and after["cumulative"] is None
    assert len(comp.layer_states) == after["layer_states"] == 0
    assert len(comp.importance_tracker.layer_scores) == after["layer_scores"] == 0
    # the compressor is reusable after the reset: the first layer again gives the same result
    comp2, infos2 = run_sequence(s)
    assert infos2[0]["compression_ratio"] == exp["per_layer"][0]["compression_ratio"]
