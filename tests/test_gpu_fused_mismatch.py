"""GPU, cfg3 size (Llama-2-7B: 32 heads of 128, S = 16384): the fused importance mode's selection against
the reference-structured W path, and the default fp32 LSE (three-way bf16 split) against the exact f32-MFMA
kernel — mismatches COUNTED and EXPLAINED.

The fused mode (K1' from Q, the prompt keys and the row LSE on MFMA; rtkv_compress_layer_qk) replaces the
materialised softmax of modified_llama.py:88-94, so its scores carry a tolerance (north_star: 1e-3
relative) and a token whose score sits within that tolerance of a class threshold (θ_h, θ_m,
dynamic_quantization.py:41-45) or of its class's selection cutoff (selective_propagation.py:93-131) may
land on the other side.  The tests assert that every label and kept-row mismatch is such a token (a label
flip whose score is within its own error of θ_h / θ_m, or a kept-row flip whose score lies between the two
paths' cutoffs of its class, widened by the tolerance) and print the counts ("MISMATCH {json}") for
DESIGN.md.  Downstream of the scores both paths are the bit-exact K2/K4."""
import json
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

S, H, D = 16384, 32, 128
TOL = 1e-3  # relative score tolerance (north_star)


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")


def _cfg():
    import rtkv
    return rtkv.CompressionConfig(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25, num_hidden_layers=32,
                                  high_precision_bits=8, medium_precision_bits=4, low_precision_bits=2)


def _inputs(dtype, seed=2024):
    """Attention that looks at the prompt by a varying amount: each head's P prompt keys share a direction e,
    and each query carries a random gain along e, so the prompt mass A (and the scores) spread over all
    three classes and the 0.8 and 0.4 budgets bind (with plain N(0, 1) queries every layer keeps every
    token and nothing is selected)."""
    import rtkv
    g = torch.Generator(device="cuda").manual_seed(seed)
    P = rtkv.prompt_length(S)
    e = torch.randn(1, H, 1, D, device="cuda", generator=g)
    e = e / e.norm(dim=-1, keepdim=True) * (0.5 * math.sqrt(D))
    # most queries lean on the prompt (gain >= 1.85 puts a late token's prompt mass above θ_h's share), so
    # about nine tokens in ten are HIGH and even layer 0's 0.8 budget (6.4 bits a token) binds
    gain = 1.0 + 3.0 * torch.rand(1, H, S, 1, device="cuda", generator=g).sqrt()
    Q = (torch.randn(1, H, S, D, device="cuda", generator=g) + gain * e).to(dtype)
    K = torch.randn(1, S, H, D, device="cuda", generator=g)
    K[:, :P] += e.permute(0, 2, 1, 3)
    K = K.reshape(1, S, H * D).to(dtype)
    V = torch.randn(1, S, H * D, device="cuda", generator=g).to(dtype)
    return Q, K, V


def _reference_w(Q, K, P):
    """The reference layer's W prompt columns: logits = Q·Kᵀ/√d in the model dtype, causal mask, softmax in
    fp32, cast back to the model dtype (modified_llama.py:88-94), computed in row chunks."""
    dt = Q.dtype
    Kh = K.view(1, S, H, D).permute(0, 2, 1, 3)
    W = torch.empty(1, H, S, P, dtype=dt, device="cuda")
    step = 1024
    for i0 in range(0, S, step):
        i1 = i0 + step
        x = torch.matmul(Q[:, :, i0:i1], Kh.transpose(2, 3)) / math.sqrt(D)
        x.masked_fill_(torch.arange(S, device="cuda")[None, :] > torch.arange(i0, i1, device="cuda")[:, None],
                       float("-inf"))
        W[:, :, i0:i1] = torch.softmax(x, dim=-1, dtype=torch.float32)[..., :P].to(dt)
        del x
    return W


def _layer(K, V, layer, W=None, Q=None, lse=None):
    import rtkv
    from rtkv import _lib as L
    cfg = _cfg()
    P = rtkv.prompt_length(S)
    ratio = rtkv.SelectiveTokenPropagator(cfg).get_layer_propagation_ratio(layer)
    p = rtkv.params_from_config(cfg, layer, P, ratio, L.EMIT_DEQUANT | L.EMIT_PACKED)
    bufs = rtkv.LayerBuffers(1, S, H * D, K.dtype, "cuda", (2, 4, 8))
    ws = rtkv.Workspace("cuda")
    res = rtkv.compress_layer(K, V, W, p, bufs, ws) if W is not None else \
        rtkv.compress_layer_qk(K, V, Q, lse, p, bufs, ws)
    res.final_stats()
    return dict(scores=bufs.scores[0].cpu().numpy().astype(np.float64), labels=bufs.labels[0].cpu().numpy(),
                mask=bufs.mask[0].cpu().numpy().astype(bool))


def _cutoffs(o):
    """Per class: the lowest kept score when the class is partly kept (its selection cutoff), else None."""
    out = []
    for c in range(3):
        inc = o["labels"] == c
        kept = inc & o["mask"]
        out.append(float(o["scores"][kept].min()) if kept.any() and kept.sum() < inc.sum() else None)
    return out


def explain(ref, new, theta_h, theta_m, tol_rel=TOL):
    """Counts of label / kept-row mismatches of `new` against `ref`, asserting each is explained: the
    scores agree within tol_rel, a label flip has θ_h or θ_m within the token's own score difference, and
    a kept-row flip of an unflipped token lies between the two paths' cutoffs of its class (widened by the
    tolerance)."""
    s0, s1 = ref["scores"], new["scores"]
    d = np.abs(s1 - s0)
    assert np.all(d <= tol_rel * np.maximum(np.abs(s0), 1e-6)), f"score error {d.max()} above {tol_rel} relative"
    tol = np.maximum(tol_rel * np.maximum(np.abs(s0), 1e-6), d)
    lab = np.nonzero(ref["labels"] != new["labels"])[0]
    for i in lab:  # on the two sides of θ_h or θ_m: the threshold lies within the token's own score error
        near = min(abs(s0[i] - theta_h), abs(s0[i] - theta_m))
        assert near <= d[i] + 1e-7, (i, s0[i], s1[i])
    T0, T1 = _cutoffs(ref), _cutoffs(new)
    keep = np.nonzero(ref["mask"] != new["mask"])[0]
    n_flip = n_cut = 0
    for i in keep:
        if ref["labels"][i] != new["labels"][i]:
            n_flip += 1
            continue
        c = int(ref["labels"][i])
        ts = [t for t in (T0[c], T1[c]) if t is not None]
        assert ts, (i, c)
        lo, hi = min(ts) - tol[i], max(ts) + tol[i]
        assert lo <= s0[i] <= hi, (i, c, s0[i], T0[c], T1[c])
        n_cut += 1
    return dict(score_max_rel_err=float((d / np.maximum(np.abs(s0), 1e-6)).max()),
                label_mismatches=int(lab.size), kept_mismatches=int(keep.size),
                kept_mismatches_by_label_flip=n_flip, kept_mismatches_between_cutoffs=n_cut,
                class_counts_ref=np.bincount(ref["labels"].astype(np.int64), minlength=3).tolist(),
                kept_ref=int(ref["mask"].sum()), kept_new=int(new["mask"].sum()),
                cutoff_ref=T0, cutoff_new=T1)


@pytest.mark.parametrize("dtype", ["float32", "float16"])
@pytest.mark.parametrize("layer", [0, 31])
def test_fused_mode_mismatches_are_threshold_ties(dtype, layer):
    import rtkv
    td = getattr(torch, dtype)
    Q, K, V = _inputs(td)
    P = rtkv.prompt_length(S)
    W = _reference_w(Q, K, P)
    ref = _layer(K, V, layer, W=W)
    del W
    lse = rtkv.attention_lse(Q, K, causal=True, k_layout="bsf")
    new = _layer(K, V, layer, Q=Q, lse=lse)
    cfg = _cfg()
    # fp32: both paths take fp32 logits, so the scores agree to the north star's 1e-3; float16: the reference
    # layer rounds its logits to fp16 before the softmax (modified_llama.py:88-94) while K1' keeps them in fp32,
    # so the W path is the less accurate side — the bound is 1e-2 and the measured error is reported
    r = explain(ref, new, cfg.theta_h, cfg.theta_m, tol_rel=TOL if dtype == "float32" else 1e-2)
    assert r["kept_ref"] < S  # the selection binds (the inputs exercise thresholds and cutoffs)
    r.update(what="fused mode (K1' on MFMA from Q, K_P, LSE) vs W path (materialised softmax)", dtype=dtype,
             layer=layer, S=S)
    print("MISMATCH " + json.dumps(r))


_EXACT_CHILD = r"""
import sys, torch, numpy as np
sys.path.insert(0, sys.argv[2])
sys.path.insert(0, sys.argv[3])
import rtkv
from test_gpu_fused_mismatch import _inputs, _layer
Q, K, V = _inputs(torch.float32)
lse = rtkv.attention_lse(Q, K, causal=True, k_layout="bsf")
o = _layer(K, V, int(sys.argv[4]), Q=Q, lse=lse)
np.savez(sys.argv[1], lse=lse.cpu().numpy(), **o)
"""


@pytest.mark.parametrize("layer", [0, 31])
def test_split_lse_layer_matches_the_exact_kernel_at_cfg3(tmp_path, layer):
    """The default fp32 LSE and K1' (three-way bf16 split on the bf16 matrix cores) against the exact
    f32-MFMA kernels (RTKV_LSE_F32_EXACT, in a child process: the knob is read once per process) on the same
    cfg3-size fp32 layer: the LSE within 1e-6 relative, and every label / kept-row difference explained as
    above (counts printed)."""
    import subprocess
    import sys
    import rtkv
    out = tmp_path / "exact.npz"
    pkg = os.path.dirname(os.path.dirname(os.path.abspath(rtkv.__file__)))
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, RTKV_LSE_F32_EXACT="1")
    subprocess.run([sys.executable, "-c", _EXACT_CHILD, str(out), pkg, here, str(layer)], env=env, check=True,
                   timeout=240)
    ex = dict(np.load(out))
    Q, K, V = _inputs(torch.float32)
    lse = rtkv.attention_lse(Q, K, causal=True, k_layout="bsf")
    np.testing.assert_allclose(lse.cpu().numpy(), ex["lse"], rtol=1e-6, atol=2e-5)
    new = _layer(K, V, layer, Q=Q, lse=lse)
    ref = dict(scores=ex["scores"], labels=ex["labels"], mask=ex["mask"])
    cfg = _cfg()
    r = explain(ref, new, cfg.theta_h, cfg.theta_m)
    r.update(what="fp32 split-bf16 LSE + K1' vs the exact f32-MFMA kernels", dtype="float32", layer=layer, S=S)
    print("MISMATCH " + json.dumps(r))
