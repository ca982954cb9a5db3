"""GPU: the fused importance mode at the reference model's precision (fp32 states, csrc/attn_f32.hip on
v_mfma_f32_16x16x4_f32) and with a padded batch (the key-padding part of the model's attention_mask
as a per-key bias).

References are torch fp32 restatements of modified_llama.py:88-94 (softmax(Q·Kᵀ/√d + attention_mask)
with the mask's finfo.min entries, so a query that sees no key gets the uniform 1/S row) and of
:124-142 (the attention over K', V' with the first S' columns of the mask).  Tolerances:
  * lse: |Δ| ≤ 2e-4 + 1e-5·|lse| (fp32 exp2/log2 and summation order); padding rows -inf exactly
  * A:   |ΔA| ≤ 2e-5 · max(A)
  * importance scores of the whole layer vs the W path fed the fp32 softmax: |Δs| ≤ 1e-3·|s|
    (north_star's rel tolerance), and K', V' bit-identical to the compressor's fused-mode outputs
  * attention output (fp32 SDPA vs the restatement): 1e-4 abs + rel."""
import numpy as np
import pytest
import torch

import rtkv_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    import rtkv
    rtkv.build()


NEG = torch.finfo(torch.float32).min


def pad_mask(B, S, left, right, device="cuda"):
    """HF-style additive fp32 mask [B, 1, S, S]: causal, plus left[b] leading and right[b] trailing
    padding keys per batch row (finfo.min entries)."""
    causal = torch.ones(S, S, dtype=torch.bool, device=device).tril()
    valid = torch.ones(B, S, dtype=torch.bool, device=device)
    for b in range(B):
        valid[b, : left[b]] = False
        if right[b]:
            valid[b, S - right[b]:] = False
    vis = causal[None] & valid[:, None, :]
    return torch.zeros(B, 1, S, S, device=device).masked_fill(~vis[:, None], NEG), valid


def ref_softmax(Q, Kh, mask_add, scale, causal=True):
    """fp32 logits + additive mask → (lse with -inf for rows that see no key, softmax rows)."""
    S = Q.shape[2]
    x = torch.einsum("bhid,bhjd->bhij", Q.float(), Kh.float()) * scale
    if mask_add is not None:
        x = x + mask_add
    elif causal:
        x = x.masked_fill(torch.ones(S, S, dtype=torch.bool, device=Q.device).triu(1), float("-inf"))
    W = torch.softmax(x, dim=-1)
    if mask_add is not None:
        seen = (mask_add > NEG / 2).expand_as(x)
        lse = torch.logsumexp(x.masked_fill(~seen, float("-inf")), dim=-1)
    else:
        lse = torch.logsumexp(x, dim=-1)
    return lse, W


def bhsd(K_bsf, Hkv, D):
    B, S, _ = K_bsf.shape
    return K_bsf.view(B, S, Hkv, D).permute(0, 2, 1, 3)


@pytest.mark.parametrize("B,H,Hkv,S,causal", [
    (1, 4, 4, 1000, True),
    (2, 8, 2, 333, True),     # GQA, ragged tiles
    (1, 4, 4, 777, False),
    (1, 2, 1, 5, True),       # tiny S
    (1, 32, 32, 2048, True),  # Llama-2-7B heads
])
def test_lse_f32(B, H, Hkv, S, causal):
    import rtkv
    D = 128
    g = torch.Generator(device="cuda").manual_seed(S + 7 * H)
    Q = torch.randn(B, H, S, D, device="cuda", generator=g) * 1.5
    K = torch.randn(B, Hkv, S, D, device="cuda", generator=g) * 1.5
    lse = rtkv.attention_lse(Q, K, causal=causal)
    ref, _ = ref_softmax(Q, K.repeat_interleave(H // Hkv, dim=1), None, D ** -0.5, causal)
    assert torch.isfinite(lse).all()
    torch.testing.assert_close(lse, ref, rtol=1e-5, atol=2e-4)
    Kbsf = K.transpose(1, 2).reshape(B, S, Hkv * D).contiguous()
    assert torch.equal(rtkv.attention_lse(Q, Kbsf, causal=causal, k_layout="bsf"), lse)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
def test_lse_and_importance_with_key_padding(dtype):
    """Left padding (batch row 1) and right padding (row 0): lse and A against the fp32 masked softmax;
    rows that see no key get lse = -inf and the uniform 1/S row (A = P/S)."""
    import rtkv
    B, H, Hkv, S, D = 2, 8, 4, 640, 128
    P = rtkv.prompt_length(S)
    g = torch.Generator(device="cuda").manual_seed(11)
    Q = torch.randn(B, H, S, D, device="cuda", generator=g).to(dtype)
    Kbsf = torch.randn(B, S, Hkv * D, device="cuda", generator=g).to(dtype)
    mask, valid = pad_mask(B, S, left=[0, 37], right=[21, 0])
    bias = torch.zeros(B, S, device="cuda").masked_fill(~valid, float("-inf"))
    lse = rtkv.attention_lse(Q, Kbsf, k_layout="bsf", key_bias=bias)
    ref_lse, W = ref_softmax(Q, bhsd(Kbsf, Hkv, D).repeat_interleave(H // Hkv, dim=1), mask, D ** -0.5)
    assert torch.isneginf(lse[1, :, :37]).all() and torch.isfinite(lse[1, :, 37:]).all()
    assert torch.isfinite(lse[0]).all()
    torch.testing.assert_close(lse, ref_lse, rtol=1e-5, atol=2e-4)
    A = rtkv.importance_qk_lse(Q, Kbsf, lse, P, key_bias=bias)
    A_ref = W[..., :P].double().mean(1).sum(-1)
    err = (A.double() - A_ref).abs().max().item()
    assert err <= 2e-5 * A_ref.abs().max().item(), err
    torch.testing.assert_close(A[1, :37], torch.full((37,), P / S, device="cuda"), rtol=1e-6, atol=0)


@pytest.mark.parametrize("B,H,Hkv,S,ratio,pad", [
    (1, 32, 32, 1024, 0.5, None),
    (2, 8, 8, 512, 0.6, ([0, 29], [0, 0])),    # left padding in batch row 1 (the reference's HF batching)
    (2, 16, 4, 768, 0.4, ([13, 0], [0, 40])),  # GQA, left + right padding
])
def test_fp32_layer_matches_w_path(B, H, Hkv, S, ratio, pad):
    """The whole layer at fp32: fused-mode scores ≈ the W path fed the fp32 masked softmax (1e-3 rel),
    downstream bit-exact with the oracle given the kernel's own A; the model-side output ≈ the fp32
    restatement of modified_llama.py:124-142 with the model's own (padded) mask."""
    import rtkv
    from rtkv.model_side import CompressedPrefillAttention
    D = 128
    g = torch.Generator(device="cuda").manual_seed(S + H)
    Q = torch.randn(B, H, S, D, device="cuda", generator=g)
    K = torch.randn(B, Hkv, S, D, device="cuda", generator=g)
    V = torch.randn(B, Hkv, S, D, device="cuda", generator=g)
    if pad is None:
        mask, valid = None, None
        bias = None
    else:
        mask, valid = pad_mask(B, S, *pad)
        bias = torch.zeros(B, S, device="cuda").masked_fill(~valid, float("-inf"))
    cfg = dict(num_hidden_layers=4, low_precision_bits=2, medium_precision_bits=4, high_precision_bits=8,
               early_layer_ratio=ratio, middle_layer_ratio=ratio, later_layer_ratio=ratio)
    comp = lambda: rtkv.RealTimePrefillCompressor(rtkv.CompressionConfig(**cfg))  # noqa: E731
    layer = CompressedPrefillAttention(comp(), H, Hkv, D, layer_idx=1)
    out, (ck, cv), info = layer(Q, K, V, attention_mask=mask)
    Sp = ck.shape[2]
    k_bsf = K.transpose(1, 2).reshape(B, S, Hkv * D).contiguous()
    v_bsf = V.transpose(1, 2).reshape(B, S, Hkv * D).contiguous()
    ids = torch.zeros(B, S, dtype=torch.long, device="cuda")
    # K'/V' are the fused-mode compressor outputs for the same inputs
    lse = rtkv.attention_lse(Q, k_bsf, k_layout="bsf", key_bias=bias)
    c1 = comp()
    k2, v2, _ = c1.compress_layer_kv_cache(k_bsf, v_bsf, None, ids, 1, query_states=Q, attention_lse=lse,
                                           key_padding_bias=bias)
    assert torch.equal(ck.transpose(1, 2).reshape(B, Sp, Hkv * D), k2)
    assert torch.equal(cv.transpose(1, 2).reshape(B, Sp, Hkv * D), v2)
    s_fused = c1.importance_tracker.layer_scores[1].numpy().reshape(B, S).astype(np.float64)
    # the W path (the reference's own input) on the fp32 masked softmax
    _, W = ref_softmax(Q, K.repeat_interleave(H // Hkv, dim=1), mask, D ** -0.5)
    c2 = comp()
    c2.compress_layer_kv_cache(k_bsf, v_bsf, W.contiguous(), ids, 1)
    s_w = c2.importance_tracker.layer_scores[1].numpy().reshape(B, S).astype(np.float64)
    rel = np.abs(s_fused - s_w) / np.abs(s_w)
    assert rel.max() <= 1e-3, rel.max()
    # downstream of A: bit-exact with the oracle's selection on the fused scores
    P = rtkv.prompt_length(S)
    labels, _ = orc.assign_precision(s_fused.astype(np.float32), 0.7, 0.3)
    sel, kept, _, _ = orc.select(s_fused.astype(np.float32), labels, (2, 4, 8), c1.propagator.get_layer_propagation_ratio(1))
    assert np.array_equal(info["propagation_info"]["selection_mask"].cpu().numpy().astype(np.uint8), sel)
    assert Sp == int(kept.max()) and P >= 1
    # the attention after compression, as the reference computes it (:124-142), in fp32
    g_ = H // Hkv
    if Sp != S:
        x = torch.einsum("bhid,bhjd->bhij", Q, ck.repeat_interleave(g_, dim=1)) * D ** -0.5
        if mask is not None:
            x = x + mask[..., :Sp]
        else:
            x = x.masked_fill(~torch.ones(S, S, dtype=torch.bool, device="cuda").tril()[:, :Sp], float("-inf"))
        ref = torch.softmax(x, dim=-1) @ cv.repeat_interleave(g_, dim=1)
    else:
        ref = W @ cv.repeat_interleave(g_, dim=1)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)
