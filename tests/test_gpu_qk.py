"""GPU: the fused importance mode (K1' on MFMA, rtkv_importance_qk_lse / rtkv_compress_layer_qk).

The mode replaces the materialised attention W = softmax(Q·Kᵀ/√d + mask) (modified_llama.py:88-94)
by Q, the P prompt keys and the row log-sum-exp.  Its reference is that softmax computed in fp32
(the reference model runs in fp32) from the same fp16/bf16 Q/K values, aggregated as
token_importance.py:21-47 does; parity is a tolerance:
  * A (prompt-attention mass per token): |ΔA| <= 2e-5 · max(A)   (fp32 exp/accumulation order)
  * importance scores: |Δs| <= 1e-3 · |s|                           (north_star: 1e-3 rel)
Downstream of A the path is the bit-exact K2/K4: given the kernel's own A, classes, selection and
quantized rows equal the oracle's bit for bit."""
import numpy as np
import pytest
import torch

import rtkv_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")


def _inputs(seed, B, H, Hkv, S, D, dtype):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    Q = torch.randn(B, H, S, D, generator=g, device="cuda").to(dtype)
    K = torch.randn(B, S, Hkv * D, generator=g, device="cuda").to(dtype)
    V = torch.randn(B, S, Hkv * D, generator=g, device="cuda").to(dtype)
    return Q, K, V


def _reference_softmax(Q, K, Hkv, causal, scale):
    """fp32 logits / LSE / prompt-column softmax of the given Q, K (chunked over query rows)."""
    B, H, S, D = Q.shape
    Kh = K.view(B, S, Hkv, D).permute(0, 2, 1, 3).float()      # [B,Hkv,S,D]
    Kh = Kh.repeat_interleave(H // Hkv, dim=1)                  # [B,H,S,D]
    lse = torch.empty(B, H, S, dtype=torch.float32, device=Q.device)
    P = max(1, min(S // 5, 128))
    Wp = torch.empty(B, H, S, P, dtype=torch.float32, device=Q.device)
    step = 1024
    for i0 in range(0, S, step):
        i1 = min(S, i0 + step)
        x = torch.matmul(Q[:, :, i0:i1].float(), Kh.transpose(2, 3)) * scale
        if causal:
            rows = torch.arange(i0, i1, device=Q.device)[:, None]
            x = x.masked_fill(torch.arange(S, device=Q.device)[None, :] > rows, float("-inf"))
        lse[:, :, i0:i1] = torch.logsumexp(x, dim=-1)
        Wp[:, :, i0:i1] = torch.softmax(x, dim=-1)[..., :P]
    return lse, Wp, P


@pytest.mark.parametrize("dtype,B,H,Hkv,S,D,causal", [
    (torch.float16, 1, 32, 32, 4096, 128, True),
    (torch.float16, 2, 8, 8, 700, 64, True),
    (torch.bfloat16, 1, 16, 4, 1000, 128, True),     # grouped-query heads
    (torch.float16, 1, 4, 4, 300, 64, False),        # P = 60 (partial MFMA tile), no mask
    (torch.bfloat16, 1, 40, 40, 2048, 128, True),    # Llama-2-13B heads
    (torch.float16, 1, 8, 8, 400, 128, True),        # head-major kernel with P = 80 (< 128 columns)
    (torch.float16, 1, 8, 8, 4000, 128, False),      # one 32-row tile per wave, rows past S in the last tile
    (torch.bfloat16, 1, 32, 8, 16384, 128, True),    # cfg3 shape: 8 tiles per wave, 2 ahead in flight
])
def test_fused_importance_matches_fp32_softmax(dtype, B, H, Hkv, S, D, causal):
    import rtkv
    Q, K, V = _inputs(5 + S, B, H, Hkv, S, D, dtype)
    scale = 1.0 / D ** 0.5
    lse, Wp, P = _reference_softmax(Q, K, Hkv, causal, scale)
    A = rtkv.importance_qk_lse(Q, K, lse, P, causal=causal)
    A_ref = Wp.double().mean(1).sum(-1)
    err = (A.double() - A_ref).abs().max().item()
    assert err <= 2e-5 * A_ref.abs().max().item(), (err, A_ref.abs().max().item())

    # the whole layer in fused mode: scores within 1e-3 rel of the fp32 reference scores, and the
    # downstream stages bit-exact given the kernel's own A
    cfg = rtkv.CompressionConfig(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25, num_hidden_layers=1,
                                 layer_weights=[1.0], high_precision_bits=8, medium_precision_bits=4,
                                 low_precision_bits=2)
    comp = rtkv.RealTimePrefillCompressor(cfg)
    k2, v2, info = comp.compress_layer_kv_cache(K, V, None, torch.zeros(B, S, dtype=torch.long, device="cuda"), 0,
                                                query_states=Q, attention_lse=lse, causal=causal)
    s_dev = comp.importance_tracker.layer_scores[0].numpy().reshape(B, S)
    s_ref = orc.importance_scores(A_ref.float().cpu().numpy(), 0, P, 0.8, 0.1, 0.1, 1.0)
    s_own = orc.importance_scores(A.cpu().numpy(), 0, P, 0.8, 0.1, 0.1, 1.0)
    assert np.array_equal(s_dev, s_own), "K2 scores differ from the oracle given the same A"
    rel = np.abs(s_dev.astype(np.float64) - s_ref) / np.abs(s_ref)
    assert rel.max() <= 1e-3, rel.max()
    labels, _ = orc.assign_precision(s_own, 0.4, 0.25)
    mask, kept, _, _ = orc.select(s_own, labels, (2, 4, 8), comp.propagator.get_layer_propagation_ratio(0))
    got_mask = info["propagation_info"]["selection_mask"].cpu().numpy().astype(np.uint8)
    assert np.array_equal(got_mask, mask)
    assert k2.shape[1] == int(kept.max())
    # dequantized rows = the oracle's per-token quantization of the kept rows
    code = {torch.float16: 1, torch.bfloat16: 2}[dtype]
    Kn = K.cpu().view(torch.int16).numpy().view(np.uint16)
    ref_k = orc.mixed_precision(Kn, code, labels, (2, 4, 8))
    for b in range(B):
        idx = np.nonzero(mask[b])[0]
        got = k2[b, : idx.size].cpu().view(torch.int16).numpy().view(np.uint16)
        assert np.array_equal(got, ref_k[b, idx])
