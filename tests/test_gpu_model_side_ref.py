"""GPU: the model-side drop-in against the REFERENCE attention layer itself.

Fixtures (tests/golden/gen_model_side.py) hold what the reference's CompressedLlamaAttention.forward
(modified_llama.py:48-168) returned, with the reference compressor set on it, for tiny fp32 Llama
layers (head_dim 128) with and without key padding: the attention output after o_proj and the
compressed cache K', V'.  Here the same states (exact by construction: q/k/v = hidden @ Wᵀ are exact
fp32 sums on any GEMM) go through rtkv.CompressedPrefillAttention — row LSE + fused-mode compression
on the GPU, the reference's attention over K', V' with the first S' columns of the model's mask — and
o_proj.

Parity:
  * importance scores: |Δs| ≤ 1e-3·|s| (north_star), and below half the fixture's selection margin
    (so classes and the selection cannot differ);
  * kept tokens, and K', V' bit for bit;
  * attention output: |Δ| ≤ 1e-4 + 1e-4·|ref| (fp32 SDPA vs the reference's fp32 matmul/softmax)."""
import json
import os

import numpy as np
import pytest
import torch

import synth

pytestmark = pytest.mark.gpu

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fixtures")
CASES = sorted(f[:-4] for f in os.listdir(FIX) if f.startswith("model_side_") and f.endswith(".npz"))


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")


def states(seed, B, S, hidden):  # the generator's recipe (gen_model_side.py: states)
    hs = np.clip(np.rint(synth.normal(seed, (B, S, hidden), 0) * 4.0), -12, 12).astype(np.float32) / 4.0
    ws = [np.clip(np.rint(synth.normal(seed, (hidden, hidden), 1 + k) * 6.0), -16, 16).astype(np.float32) / 128.0
          for k in range(4)]
    return hs, ws


def test_fixture_inventory():
    assert len(CASES) >= 4


@pytest.mark.parametrize("name", CASES)
def test_model_side_matches_reference_layer(name):
    import rtkv
    from rtkv.model_side import CompressedPrefillAttention
    z = np.load(os.path.join(FIX, name + ".npz"))
    spec = json.loads(str(z["spec"]))
    assert not spec["rope_applied"]
    B, S, nh, hidden, layer = spec["B"], spec["S"], spec["heads"], spec["hidden"], spec["layer"]
    D = 128
    hs, (wq, wk, wv, wo) = (states(spec["seed"], B, S, hidden))
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    h = dev(hs)
    q = (h @ dev(wq).t()).view(B, S, nh, D).transpose(1, 2)
    k = (h @ dev(wk).t()).view(B, S, nh, D).transpose(1, 2)
    v = (h @ dev(wv).t()).view(B, S, nh, D).transpose(1, 2)
    valid = torch.ones(B, S, dtype=torch.bool)
    for b in range(B):
        valid[b, : spec["left"][b]] = False
        if spec["right"][b]:
            valid[b, S - spec["right"][b]:] = False
    vis = torch.ones(S, S, dtype=torch.bool).tril()[None] & valid[:, None, :]
    mask = torch.zeros(B, 1, S, S).masked_fill(~vis[:, None], torch.finfo(torch.float32).min).cuda()
    comp = rtkv.RealTimePrefillCompressor(rtkv.CompressionConfig(num_hidden_layers=4, **spec["config"]))
    layer_mod = CompressedPrefillAttention(comp, nh, nh, D, layer_idx=layer)
    ids = torch.zeros(B, S, dtype=torch.long, device="cuda")
    out, (ck, cv), info = layer_mod(q, k, v, ids, attention_mask=mask)
    # scores: within the north star's tolerance and well inside the selection margins
    s = comp.importance_tracker.layer_scores[layer].numpy().reshape(B, S).astype(np.float64)
    s_ref = z["scores"].astype(np.float64)
    d = np.abs(s - s_ref)
    assert (d <= 1e-3 * np.abs(s_ref)).all(), d.max()
    assert d.max() < 0.5 * min(spec["margin_theta"], spec["margin_select"]), (d.max(), spec)
    # the same tokens kept, and K', V' bit for bit
    assert np.array_equal(info["propagation_info"]["selection_mask"].cpu().numpy().astype(bool), z["kept"])
    assert ck.shape == z["k_out"].shape and cv.shape == z["v_out"].shape
    assert np.array_equal(ck.cpu().numpy().view(np.uint32), z["k_out"].view(np.uint32))
    assert np.array_equal(cv.cpu().numpy().view(np.uint32), z["v_out"].view(np.uint32))
    # the layer's output after o_proj
    o = out.transpose(1, 2).reshape(B, S, hidden) @ dev(wo).t()
    torch.testing.assert_close(o.cpu(), torch.from_numpy(z["attn_output"]), rtol=1e-4, atol=1e-4)
