"""Model-side drop-in for the compression step of CompressedLlamaAttention.

The reference attention layer (src/models/modified_llama.py:96-149) materialises
softmax(Q·Kᵀ/√d + mask) as a [B, H, S, S] tensor only to hand it to compress_layer_kv_cache, then
recomputes the attention over the compressed keys.  `CompressedPrefillAttention` keeps the same
three steps without that tensor:

1. the row log-sum-exp of the prefill softmax, on MFMA (rtkv_attention_lse, csrc/attn_lse.hip);
2. the compression in the fused importance mode: Q, the prompt keys and the lse give the
   prompt-attention mass (rtkv_compress_layer_qk, K1' on MFMA), then the usual selection and
   quantization (K2, K4) — K', V' and the packed codes as in the reference layer;
3. the attention output the reference computes after compression (modified_llama.py:124-142):
   over the compressed keys when tokens were dropped, with the reference's mask handling — the
   *first* S' columns of the causal mask (:131-134), or the causal mask over
   the kept positions when `position_mask=True` (the fix; a query before the first kept position
   gets a zero output) — else over the original keys with the
   compressed values.  This step is PyTorch's fused scaled-dot-product attention (the model's own
   attention, not part of the compression path).

Inputs are the post-RoPE states the reference layer has at :64-75, in its [B, heads, S, D] layout.

Limits at this boundary (checked, ValueError): the states are float16 or bfloat16 with head_dim 64 or
128 (the MFMA LSE and K1' kernels), and the model's attention_mask, when given, must be the plain
causal mask — a padded batch (padding columns in the mask, modified_llama.py:90-91) is rejected
rather than silently scored as unpadded.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as Fn

from .engine import attention_lse


class CompressedPrefillAttention:
    """compressor: a RealTimePrefillCompressor (the reference's set_compressor, :40-42)."""

    def __init__(self, compressor, num_heads: int, num_kv_heads: int, head_dim: int, layer_idx: int,
                 position_mask: bool = False):
        self.compressor = compressor
        self.num_heads = num_heads
        self.num_kv_heads = num_kv_heads
        self.head_dim = head_dim
        self.layer_idx = layer_idx
        self.position_mask = position_mask

    def __call__(self, query_states: torch.Tensor, key_states: torch.Tensor, value_states: torch.Tensor,
                 input_ids: Optional[torch.Tensor] = None,
                 attention_mask: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, Tuple[torch.Tensor, torch.Tensor], Dict]:
        """query [B,H,S,D], key/value [B,Hkv,S,D] (post-RoPE) → (attn_output [B,H,S,D] before o_proj,
        (K' [B,Hkv,S',D], V' [B,Hkv,S',D]) for the cache, compression_info).  attention_mask: the
        model's additive [B, 1, S, S] mask (optional; only the causal mask is accepted)."""
        B, H, S, D = query_states.shape
        Hkv = key_states.shape[1]
        if H != self.num_heads or Hkv != self.num_kv_heads or D != self.head_dim:
            raise ValueError("state shapes do not match the layer's head configuration")
        if query_states.dtype not in (torch.float16, torch.bfloat16) or D not in (64, 128):
            raise ValueError(f"CompressedPrefillAttention needs float16/bfloat16 states with head_dim 64 or 128 "
                             f"(got {query_states.dtype}, head_dim {D}); fp32 models use the reference attention "
                             f"with RealTimePrefillCompressor.compress_layer_kv_cache")
        if attention_mask is not None:
            m = attention_mask[..., :S, :S]
            causal = torch.ones(S, S, dtype=torch.bool, device=m.device).tril()
            if m.dim() != 4 or not bool(torch.equal((m >= 0).expand(B, 1, S, S), causal.expand(B, 1, S, S))):
                raise ValueError("attention_mask is not the plain causal mask (padded batches are not supported by "
                                 "the fused importance mode)")
        Q = query_states.contiguous()
        # [B, S, Hkv·D] keys/values as the reference reshapes them for the compressor (:104-107)
        k_bsf = key_states.transpose(1, 2).reshape(B, S, Hkv * D).contiguous()
        v_bsf = value_states.transpose(1, 2).reshape(B, S, Hkv * D).contiguous()
        lse = attention_lse(Q, k_bsf, causal=True, k_layout="bsf")
        ids = input_ids if input_ids is not None else torch.zeros(B, S, dtype=torch.long, device=Q.device)
        k2, v2, info = self.compressor.compress_layer_kv_cache(k_bsf, v_bsf, None, ids, self.layer_idx,
                                                               query_states=Q, attention_lse=lse)
        Sp = k2.shape[1]
        ck = k2.view(B, Sp, Hkv, D).transpose(1, 2)
        cv = v2.view(B, Sp, Hkv, D).transpose(1, 2)
        g = H // Hkv
        if Sp != S:
            keys, vals = ck, cv
            if self.position_mask:
                # causal over the kept positions: key j (source token kept_index[b, j]) ≤ query i
                # (sync-free: each kept token lands at its rank among the row's kept tokens; dropped
                # tokens all land in a spare column that is cut off)
                pos = info["propagation_info"]["selection_mask"]
                rank = pos.long().cumsum(-1) - 1
                tgt = torch.where(pos, rank, torch.full_like(rank, Sp))
                kp = torch.full((B, Sp + 1), S, dtype=torch.long, device=Q.device)
                kp.scatter_(1, tgt, torch.arange(S, device=Q.device).expand(B, S))
                kept_pos = kp[:, :Sp]
                mask = kept_pos[:, None, None, :] <= torch.arange(S, device=Q.device)[None, None, :, None]
                # a query before the first kept position sees no key: its output is zero
                empty = ~mask.any(dim=-1, keepdim=True)
                mask = mask | empty
            else:
                # the reference: the first S' columns of the causal mask (:131-134)
                mask = torch.ones(S, S, dtype=torch.bool, device=Q.device).tril()[:, :Sp][None, None]
        else:
            keys, vals = key_states, cv  # original weights with the compressed values (:139-140)
            mask = None
        if g > 1:
            keys = keys.repeat_interleave(g, dim=1)
            vals = vals.repeat_interleave(g, dim=1)
        if mask is None:
            out = Fn.scaled_dot_product_attention(Q, keys, vals, is_causal=True)
        else:
            out = Fn.scaled_dot_product_attention(Q, keys, vals, attn_mask=mask)
            if Sp != S and self.position_mask:
                out = out.masked_fill(empty, 0.0)
        return out, (ck, cv), info
