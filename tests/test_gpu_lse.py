"""GPU: the attention row log-sum-exp (rtkv_attention_lse, csrc/attn_lse.hip) against a torch fp32
logsumexp of the masked scores, and the fused importance mode fed by it.

The kernel multiplies fp16/bf16 Q·K on MFMA with fp32 accumulation (fp32 Q·K: three bf16 parts per
operand, six part products — fp32-accurate) and sums exp2 in fp32, so the tolerance is
|Δlse| ≤ 2e-4 + 1e-5·|lse| (summation order and the hardware exp2/log2).  Cases: causal
and full attention, head_dim 64 and 128, GQA (H / Hkv = 4), S not a multiple of the 64-row tiles,
tiny S, batch 2, both layouts of K."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    import rtkv
    rtkv.build()


def ref_lse(Q, K, causal, scale):
    """Q [B,H,S,D], K [B,Hkv,S,D] → lse [B,H,S] in fp32."""
    B, H, S, D = Q.shape
    g = H // K.shape[1]
    Kf = K.float().repeat_interleave(g, dim=1)
    s = torch.einsum("bhid,bhjd->bhij", Q.float(), Kf) * scale
    if causal:
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=Q.device).triu(1), float("-inf"))
    return torch.logsumexp(s, dim=-1)


CASES = [
    # B, H, Hkv, S, D, dtype, causal
    (1, 4, 4, 1000, 128, torch.float16, True),
    (2, 8, 2, 333, 64, torch.bfloat16, True),
    (1, 4, 4, 777, 128, torch.bfloat16, False),
    (1, 2, 2, 64, 128, torch.float16, True),
    (1, 2, 1, 5, 64, torch.float16, True),
    (1, 32, 32, 4096, 128, torch.float16, True),
    # fp32 states: the split-bf16 kernel (three bf16 parts per operand, six products; attn_f32.hip)
    (1, 4, 4, 1000, 128, torch.float32, True),
    (2, 8, 2, 333, 128, torch.float32, True),
    (1, 4, 4, 777, 128, torch.float32, False),
    (1, 2, 2, 64, 128, torch.float32, True),
    (1, 32, 32, 4096, 128, torch.float32, True),
]


@pytest.mark.parametrize("B,H,Hkv,S,D,dtype,causal", CASES, ids=lambda v: str(v).replace("torch.", ""))
def test_attention_lse(B, H, Hkv, S, D, dtype, causal):
    import rtkv
    g = torch.Generator(device="cuda").manual_seed(S * 31 + H)
    Q = (torch.randn(B, H, S, D, device="cuda", generator=g) * 1.5).to(dtype)
    K = (torch.randn(B, Hkv, S, D, device="cuda", generator=g) * 1.5).to(dtype)
    scale = 1.0 / D ** 0.5
    lse = rtkv.attention_lse(Q, K, causal=causal)
    ref = ref_lse(Q, K, causal, scale)
    assert torch.isfinite(lse).all()
    torch.testing.assert_close(lse, ref, rtol=1e-5, atol=2e-4)
    # the [B, S, Hkv*D] layout of the compressor's key input gives the same result
    Kbsf = K.transpose(1, 2).reshape(B, S, Hkv * D).contiguous()
    assert torch.equal(rtkv.attention_lse(Q, Kbsf, causal=causal, k_layout="bsf"), lse)


def test_fused_importance_from_own_lse():
    """K1' fed by rtkv_attention_lse == K1' fed by the torch fp32 lse (to the lse tolerance)."""
    import rtkv
    B, H, S, D, P = 1, 8, 2048, 128, 128
    g = torch.Generator(device="cuda").manual_seed(5)
    Q = torch.randn(B, H, S, D, device="cuda", generator=g).half()
    K = torch.randn(B, H, S, D, device="cuda", generator=g).half()
    lse = rtkv.attention_lse(Q, K)
    ref = ref_lse(Q, K, True, 1.0 / D ** 0.5).contiguous()
    Kbsf = K.transpose(1, 2).reshape(B, S, H * D).contiguous()
    A = rtkv.importance_qk_lse(Q, Kbsf, lse, P)
    A_ref = rtkv.importance_qk_lse(Q, Kbsf, ref, P)
    torch.testing.assert_close(A, A_ref, rtol=1e-3, atol=1e-6)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32])
def test_overflow_rows_take_the_fixup_pass(dtype):
    """The 32x32 kernel sums against each row's first logit unchecked; a later logit ~180 log2 units
    above it overflows the sum, and the fix-up pass must recompute those rows (attn_lse32.hip).  fp32
    (the split-bf16 kernel) raises its reference max lazily instead: the same rows must stay finite."""
    import rtkv
    B, H, S, D = 1, 4, 1024, 128
    g = torch.Generator(device="cuda").manual_seed(9)
    Q = torch.randn(B, H, S, D, device="cuda", generator=g)
    K = torch.randn(B, H, S, D, device="cuda", generator=g)
    K[:, :, 700] = 4.0   # one key aligned with the boosted queries: q·k·scale ≈ 181 → 261 in log2 units
    Q[:, :, 800:900] = 4.0
    Q, K = Q.to(dtype), K.to(dtype)
    lse = rtkv.attention_lse(Q, K)
    ref = ref_lse(Q, K, True, 1.0 / D ** 0.5)
    assert torch.isfinite(lse).all()
    torch.testing.assert_close(lse, ref, rtol=1e-5, atol=2e-4)


def test_rejects_unsupported():
    import rtkv
    Q = torch.zeros(1, 2, 64, 96, device="cuda", dtype=torch.float16)
    with pytest.raises(RuntimeError, match="head_dim"):
        rtkv.attention_lse(Q, Q)


_EXACT_CHILD = r"""
import sys, torch
sys.path.insert(0, sys.argv[2])
import rtkv
g = torch.Generator(device="cuda").manual_seed(17)
B, H, Hkv, S, D = 1, 8, 2, 1500, 128
Q = torch.randn(B, H, S, D, device="cuda", generator=g) * 1.5
K = torch.randn(B, Hkv, S, D, device="cuda", generator=g) * 1.5
torch.save({"lse": rtkv.attention_lse(Q, K, causal=True).cpu(), "Q": Q.cpu(), "K": K.cpu()}, sys.argv[1])
"""


def test_fp32_split_lse_matches_the_exact_f32_kernel(tmp_path):
    """The split-bf16 fp32 LSE (six bf16 part products) against the exact f32-MFMA kernel
    (RTKV_LSE_F32_EXACT, run in a child process: the knob is read once per process) on the same
    inputs: fp32-accurate, i.e. far inside the 2e-4 tolerance against torch."""
    import os
    import subprocess
    import sys
    import rtkv
    out = tmp_path / "exact.pt"
    pkg = os.path.dirname(os.path.dirname(os.path.abspath(rtkv.__file__)))
    env = dict(os.environ, RTKV_LSE_F32_EXACT="1")
    subprocess.run([sys.executable, "-c", _EXACT_CHILD, str(out), pkg], env=env, check=True, timeout=120)
    d = torch.load(out, weights_only=True)
    lse = rtkv.attention_lse(d["Q"].cuda(), d["K"].cuda(), causal=True).cpu()
    assert torch.isfinite(lse).all()
    torch.testing.assert_close(lse, d["lse"], rtol=1e-6, atol=2e-5)
