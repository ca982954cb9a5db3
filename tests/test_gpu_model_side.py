"""GPU: the model-side drop-in (rtkv.model_side.CompressedPrefillAttention).

Checks, per case: the compressed K'/V' are exactly what the compressor returns in the fused
importance mode for the same Q/K/V (the lse coming from rtkv_attention_lse); the attention output
matches a torch fp32 restatement of modified_llama.py:124-142 over those K'/V' — the first S' causal
mask columns when tokens were dropped (the reference's behaviour), the causal mask over the kept
positions with position_mask=True, and the original keys with the compressed values when nothing
was dropped.  Tolerance: the output comes from fp16/bf16 SDPA, |Δ| ≤ t + t·|ref| with t = 3e-3
(fp16) or 1.6e-2 (bf16, 8-bit significand)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    import rtkv
    rtkv.build()


def compressor(ratio, bits=(8, 8, 8)):
    import rtkv
    cfg = rtkv.CompressionConfig(num_hidden_layers=4, low_precision_bits=bits[0], medium_precision_bits=bits[1],
                                 high_precision_bits=bits[2], early_layer_ratio=ratio, middle_layer_ratio=ratio,
                                 later_layer_ratio=ratio)
    return rtkv.RealTimePrefillCompressor(cfg)


def ref_attention(Q, keys, vals, mask):
    """fp32 softmax(Q·Kᵀ/√d masked)·V with GQA by head repetition; mask [B|1, 1, S, S'] bool."""
    H, D = Q.shape[1], Q.shape[3]
    g = H // keys.shape[1]
    k = keys.float().repeat_interleave(g, dim=1)
    v = vals.float().repeat_interleave(g, dim=1)
    s = torch.einsum("bhid,bhjd->bhij", Q.float(), k) / D ** 0.5
    s = s.masked_fill(~mask, float("-inf"))
    return torch.softmax(s, dim=-1) @ v


CASES = [
    # B, H, Hkv, S, dtype, ratio, position_mask
    (1, 8, 8, 512, torch.float16, 0.5, False),
    (1, 8, 8, 512, torch.float16, 0.5, True),
    (2, 32, 8, 384, torch.bfloat16, 0.6, False),
    (1, 8, 8, 256, torch.float16, 1.0, False),
    (2, 16, 4, 640, torch.bfloat16, 0.5, True),   # ragged kept counts across the batch, GQA
]


@pytest.mark.parametrize("B,H,Hkv,S,dtype,ratio,pmask", CASES, ids=lambda v: str(v).replace("torch.", ""))
def test_compressed_prefill_attention(B, H, Hkv, S, dtype, ratio, pmask):
    import rtkv
    from rtkv.model_side import CompressedPrefillAttention
    D = 128
    g = torch.Generator(device="cuda").manual_seed(S + H)
    Q = torch.randn(B, H, S, D, device="cuda", generator=g).to(dtype)
    K = torch.randn(B, Hkv, S, D, device="cuda", generator=g).to(dtype)
    V = torch.randn(B, Hkv, S, D, device="cuda", generator=g).to(dtype)
    layer = CompressedPrefillAttention(compressor(ratio), H, Hkv, D, layer_idx=1, position_mask=pmask)
    out, (ck, cv), info = layer(Q, K, V)
    Sp = ck.shape[2]
    assert ck.shape == (B, Hkv, Sp, D) and cv.shape == (B, Hkv, Sp, D) and out.shape == (B, H, S, D)
    # K'/V' are the fused-mode compressor outputs for the same inputs
    k_bsf = K.transpose(1, 2).reshape(B, S, Hkv * D).contiguous()
    v_bsf = V.transpose(1, 2).reshape(B, S, Hkv * D).contiguous()
    lse = rtkv.attention_lse(Q, k_bsf, k_layout="bsf")
    k2, v2, _ = compressor(ratio).compress_layer_kv_cache(k_bsf, v_bsf, None, torch.zeros(B, S, dtype=torch.long,
                                                                                         device="cuda"),
                                                          1, query_states=Q, attention_lse=lse)
    assert torch.equal(ck.transpose(1, 2).reshape(B, Sp, Hkv * D), k2)
    assert torch.equal(cv.transpose(1, 2).reshape(B, Sp, Hkv * D), v2)
    causal = torch.ones(S, S, dtype=torch.bool, device="cuda").tril()
    if Sp == S:
        ref = ref_attention(Q, K, cv, causal[None, None])
    elif pmask:
        sel = info["propagation_info"]["selection_mask"]
        kp = torch.full((B, Sp), S, dtype=torch.long, device="cuda")  # padding rows: never visible
        for b in range(B):
            idx = sel[b].nonzero().flatten()
            kp[b, : idx.numel()] = idx
        mask = kp[:, None, None, :] <= torch.arange(S, device="cuda")[None, None, :, None]
        ref = ref_attention(Q, ck, cv, mask).nan_to_num(0.0)  # queries with no visible kept key: 0
    else:
        assert Sp < S
        ref = ref_attention(Q, ck, cv, causal[:, :Sp][None, None])
    tol = 3e-3 if dtype == torch.float16 else 1.6e-2  # one rounding of the output to the dtype
    torch.testing.assert_close(out.float(), ref, rtol=tol, atol=tol)


def test_attention_mask_and_dtype_limits():
    """The plain causal mask is accepted (same output as no mask); masks that are not causal + key
    padding, a padded mask at head_dim 64 and fp32 states at head_dim 64 are rejected at the boundary."""
    from rtkv.model_side import CompressedPrefillAttention
    B, H, S, D = 2, 8, 256, 64
    g = torch.Generator(device="cuda").manual_seed(5)
    Q, K, V = (torch.randn(B, H, S, D, device="cuda", generator=g).half() for _ in range(3))
    layer = CompressedPrefillAttention(compressor(0.5), H, H, D, layer_idx=1)
    out0, _, _ = layer(Q, K, V)
    neg = torch.finfo(torch.float16).min
    causal = torch.zeros(S, S, device="cuda").masked_fill(~torch.ones(S, S, dtype=torch.bool, device="cuda").tril(), neg)
    mask = causal[None, None].expand(B, 1, S, S).half()
    out1, _, _ = layer(Q, K, V, attention_mask=mask)
    assert torch.equal(out0, out1)
    padded = mask.clone()
    padded[1, :, :, :7] = neg  # left padding of batch row 1
    with pytest.raises(ValueError, match="head_dim 128"):
        layer(Q, K, V, attention_mask=padded)
    window = mask.clone()
    window[:, :, 100:, :3] = neg  # a sliding-window-like mask: not causal + key padding
    with pytest.raises(ValueError, match="causal"):
        layer(Q, K, V, attention_mask=window)
    odd = mask.clone()
    odd[0, 0, 5, 0] = -3.0  # an additive bias that is neither 0 nor a mask value
    with pytest.raises(ValueError, match="0 or"):
        layer(Q, K, V, attention_mask=odd)
    with pytest.raises(ValueError, match="head_dim 128"):
        layer(Q.float(), K.float(), V.float())
