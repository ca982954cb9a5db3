#!/usr/bin/env python3
"""Model-side fixtures: run the REFERENCE attention layer itself,
CompressedLlamaAttention.forward (src/models/modified_llama.py:48-168), with the reference compressor
set on it, on a tiny fp32 Llama config, and record what it returns: the attention output (after
o_proj) and the compressed cache (K', V').

Run in the build container only (imports /root/reference and transformers):

    python tests/golden/gen_model_side.py       # writes tests/golden/fixtures/model_side_*.npz

Inputs are exact by construction so that any GEMM order reproduces the states bit for bit: hidden
states are multiples of 2^-2 in [-3, 3] and projection weights multiples of 2^-7 in [-16, 16]·2^-7
(synth.py's portable generator), so q/k/v = hidden @ Wᵀ are exact fp32 sums on any machine.  With the
transformers in this image the reference module has no `rotary_emb` attribute, so its forward applies
no RoPE (modified_llama.py:72-74); the fixture records that, and the GPU test feeds the same
projections.  Each case records the selection margins of the reference scores (distance of every
score to θ_h/θ_m and to the kept/dropped boundary of its class), so the test can tell a tolerance-
level difference of the fused-mode scores from a real one.
"""
from __future__ import annotations

import json
import os
import sys

os.environ.setdefault("ATEN_CPU_CAPABILITY", "avx2")
os.environ.setdefault("OMP_NUM_THREADS", "1")

import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("RTKV_REFERENCE", "/root/reference")
OUT = os.path.join(HERE, "fixtures")
sys.path.insert(0, HERE)
sys.path.insert(0, REF)
sys.path.insert(0, os.path.join(REF, "src"))

import synth  # noqa: E402
from configs.base_config import CompressionConfig  # noqa: E402
from src.compression.unified_compressor import RealTimePrefillCompressor  # noqa: E402
from models.modified_llama import CompressedLlamaAttention  # noqa: E402
from transformers import LlamaConfig  # noqa: E402

torch.set_num_threads(1)

COV = dict(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25, high_precision_bits=8,
           medium_precision_bits=4, low_precision_bits=2, early_layer_ratio=0.8, middle_layer_ratio=0.6,
           later_layer_ratio=0.4)

CASES = [
    dict(name="model_side_b1", B=1, S=96, heads=4, left=[0], right=[0], seed=7101, layer=2),
    dict(name="model_side_b2_pad", B=2, S=96, heads=4, left=[0, 11], right=[7, 0], seed=7102, layer=3),
    dict(name="model_side_b2_pad_l3", B=2, S=128, heads=2, left=[5, 0], right=[0, 0], seed=7103, layer=3),
    dict(name="model_side_b2_pad_keepall", B=2, S=96, heads=4, left=[0, 11], right=[7, 0], seed=7104, layer=1),
]


def states(seed, B, S, hidden):
    """Exact-GEMM inputs: hidden (multiples of 2^-2) and q/k/v/o weights (multiples of 2^-7)."""
    hs = np.clip(np.rint(synth.normal(seed, (B, S, hidden), 0) * 4.0), -12, 12).astype(np.float32) / 4.0
    ws = []
    for k in range(4):
        w = np.clip(np.rint(synth.normal(seed, (hidden, hidden), 1 + k) * 6.0), -16, 16).astype(np.float32)
        ws.append(w / 128.0)
    return hs, ws


def pad_mask(B, S, left, right):
    valid = np.ones((B, S), bool)
    for b in range(B):
        valid[b, : left[b]] = False
        if right[b]:
            valid[b, S - right[b]:] = False
    vis = np.tril(np.ones((S, S), bool))[None] & valid[:, None, :]
    m = np.where(vis, 0.0, np.finfo(np.float32).min).astype(np.float32)[:, None]
    return m, valid


def margins(scores, cfg, kept_mask):
    """Smallest |Δ| between a score and θ_h/θ_m, and between kept and dropped scores of one class."""
    s = scores.astype(np.float64)
    th = min(np.abs(s - cfg["theta_h"]).min(), np.abs(s - cfg["theta_m"]).min())
    cls = np.where(s > cfg["theta_h"], 2, np.where(s > cfg["theta_m"], 1, 0))
    sel = np.inf
    for b in range(s.shape[0]):
        for c in range(3):
            k = s[b][(cls[b] == c) & kept_mask[b]]
            d = s[b][(cls[b] == c) & ~kept_mask[b]]
            if k.size and d.size:
                sel = min(sel, k.min() - d.max())
    return float(th), float(sel)


def main():
    os.makedirs(OUT, exist_ok=True)
    for c in CASES:
        B, S, nh = c["B"], c["S"], c["heads"]
        hidden = nh * 128
        hs, (wq, wk, wv, wo) = states(c["seed"], B, S, hidden)
        mask, valid = pad_mask(B, S, c["left"], c["right"])
        lc = LlamaConfig(hidden_size=hidden, num_attention_heads=nh, num_key_value_heads=nh,
                         intermediate_size=2 * hidden, num_hidden_layers=4, vocab_size=128,
                         attention_bias=False)
        attn = CompressedLlamaAttention(lc, layer_idx=c["layer"]).eval()
        with torch.no_grad():
            for lin, w in ((attn.q_proj, wq), (attn.k_proj, wk), (attn.v_proj, wv), (attn.o_proj, wo)):
                lin.weight.copy_(torch.from_numpy(w))
        rope = getattr(attn, "rotary_emb", None) is not None
        comp = RealTimePrefillCompressor(CompressionConfig(num_hidden_layers=4, **COV))
        attn.set_compressor(comp)
        ids = torch.zeros(B, S, dtype=torch.long)
        with torch.no_grad():
            outs = attn(hidden_states=torch.from_numpy(hs), attention_mask=torch.from_numpy(mask),
                        use_cache=True, input_ids=ids)
        out = outs[0].numpy()
        ck, cv = (t.numpy() for t in outs[-1])
        assert c["layer"] in comp.layer_states, "the reference layer fell back (compression failed)"
        info = comp.layer_states[c["layer"]]
        kept = info["propagation_info"]["selection_mask"].numpy().astype(bool)
        scores = comp.importance_tracker.layer_scores[c["layer"]].numpy().reshape(B, S)
        m_th, m_sel = margins(scores, COV, kept)
        spec = dict(c, hidden=hidden, config=COV, rope_applied=bool(rope), kept=int(ck.shape[2]),
                    margin_theta=m_th, margin_select=m_sel,
                    states="hidden multiples of 2^-2 in [-3,3] (synth.normal(seed, (B,S,hidden), 0)*4, rint, clip "
                           "±12, /4); W_q,k,v,o multiples of 2^-7 (synth.normal(seed, (hidden,hidden), 1..4)*6, rint, "
                           "clip ±16, /128)",
                    mask="causal + key padding, float32 min entries, [B,1,S,S]")
        np.savez_compressed(os.path.join(OUT, c["name"] + ".npz"), attn_output=out, k_out=ck, v_out=cv,
                            scores=scores, kept=kept, spec=np.array(json.dumps(spec)))
        print(c["name"], "S'", ck.shape[2], "of", S, "rope", rope, "margins θ %.3g sel %.3g" % (m_th, m_sel),
              flush=True)


if __name__ == "__main__":
    main()
