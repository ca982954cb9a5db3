"""Model-side drop-in for the compression step of CompressedLlamaAttention.

The reference attention layer (src/models/modified_llama.py:96-149) materialises
softmax(Q·Kᵀ/√d + mask) as a [B, H, S, S] tensor only to hand it to compress_layer_kv_cache, then
recomputes the attention over the compressed keys.  `CompressedPrefillAttention` keeps the same
three steps without that tensor:

1. the row log-sum-exp of the prefill softmax, on MFMA (rtkv_attention_lse, csrc/attn_lse.hip; fp32
   states on the f32 MFMA, csrc/attn_f32.hip);
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

Masks: the model's additive attention_mask [B, 1, S, S] (modified_llama.py:90-91) is accepted when it
is the causal mask plus a key-padding mask (HF's left or right padding: every entry 0 or at most
finfo.min/2, and a key masked for one query masked for all).  Its padding part becomes a per-key bias
(0 / -inf) that the LSE and K1' kernels apply, and the attention after compression uses the model's
own mask exactly as the reference does — its first S' columns (:131-134), or the whole mask when
nothing was dropped.  A query row that sees no key at all (a padding row) has lse = -inf and the
uniform 1/S softmax row the reference's all-masked row has (exact for an fp32 mask, whose finfo.min
absorbs every logit).

Limits (checked, ValueError): float32, float16 or bfloat16 states; head_dim 128 (or 64 for
float16/bfloat16 without padding); S a multiple of 4 with a padding mask; any other mask is
rejected rather than silently scored as something else.
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
        model's additive [B, 1, S, S] mask (optional; causal, with or without key padding)."""
        B, H, S, D = query_states.shape
        Hkv = key_states.shape[1]
        if H != self.num_heads or Hkv != self.num_kv_heads or D != self.head_dim:
            raise ValueError("state shapes do not match the layer's head configuration")
        dt = query_states.dtype
        if dt not in (torch.float32, torch.float16, torch.bfloat16) or D not in (64, 128) or \
                (dt == torch.float32 and D != 128):
            raise ValueError(f"CompressedPrefillAttention needs float32/float16/bfloat16 states with head_dim 128 "
                             f"(64 for float16/bfloat16); got {dt}, head_dim {D}")
        key_bias, valid_key = None, None
        if attention_mask is not None:
            key_bias, valid_key = split_attention_mask(attention_mask, B, S)
            if key_bias is not None and (D != 128 or S % 4):
                raise ValueError("a padded attention_mask needs head_dim 128 and S % 4 == 0")
        Q = query_states.contiguous()
        # [B, S, Hkv·D] keys/values as the reference reshapes them for the compressor (:104-107)
        k_bsf = key_states.transpose(1, 2).reshape(B, S, Hkv * D).contiguous()
        v_bsf = value_states.transpose(1, 2).reshape(B, S, Hkv * D).contiguous()
        lse = attention_lse(Q, k_bsf, causal=True, k_layout="bsf", key_bias=key_bias)
        ids = input_ids if input_ids is not None else torch.zeros(B, S, dtype=torch.long, device=Q.device)
        k2, v2, info = self.compressor.compress_layer_kv_cache(k_bsf, v_bsf, None, ids, self.layer_idx,
                                                               query_states=Q, attention_lse=lse,
                                                               key_padding_bias=key_bias)
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
                if valid_key is not None:  # kept padding tokens stay masked
                    vk = torch.cat([valid_key, valid_key.new_zeros(B, 1)], 1).gather(1, kept_pos)
                    mask = mask & vk[:, None, None, :]
                # a query that sees no key (before the first kept position, or padding): zero output
                empty = ~mask.any(dim=-1, keepdim=True)
                mask = mask | empty
            elif key_bias is not None:
                # the reference: the first S' columns of the model's (padded) mask (:131-134)
                mask = attention_mask[..., :S, :Sp].to(Q.dtype)
            else:
                # the first S' columns of the causal mask: tril(ones(S, S'))[i, j] = j <= i, which is
                # SDPA's is_causal for S queries over S' < S keys (upper-left aligned), so the fused
                # causal kernels run instead of a masked one
                mask = None
        else:
            keys, vals = key_states, cv  # original weights with the compressed values (:139-140)
            mask = None if attention_mask is None or key_bias is None else attention_mask[..., :S, :S].to(Q.dtype)
        if g > 1:
            keys = keys.repeat_interleave(g, dim=1)
            vals = vals.repeat_interleave(g, dim=1)
        if mask is None:  # causal: over S keys, or upper-left over the S' kept keys (see above)
            out = Fn.scaled_dot_product_attention(Q, keys, vals, is_causal=True)
        else:
            out = Fn.scaled_dot_product_attention(Q, keys, vals, attn_mask=mask)
            if Sp != S and self.position_mask:
                out = out.masked_fill(empty, 0.0)
            elif mask.dtype != torch.bool:
                # a query row the model's mask hides every key from (padding): the reference's softmax
                # of equal logits is uniform, so its output is the mean of the values (SDPA kernels may
                # return zeros for such rows).  Query i sees key j < n_keys iff j <= i and key j is valid
                # (the validated mask): blind iff no valid key among the first min(i + 1, n_keys).
                n_keys = keys.shape[2]
                seen = valid_key[:, :n_keys].long().cumsum(-1)                       # [B, n_keys]
                last = torch.arange(S, device=Q.device).clamp(max=n_keys - 1)
                blind = (seen[:, last] == 0)[:, None, :, None]                      # [B, 1, S, 1]
                out = torch.where(blind, vals.mean(dim=2, keepdim=True).to(out.dtype), out)
        return out, (ck, cv), info


def split_attention_mask(attention_mask: torch.Tensor, B: int, S: int):
    """The model's additive mask [B or 1, 1, S, >=S] → (key_bias, valid_key): None, None for the plain
    causal mask; else the fp32 [B, S] key bias (0 real key, -inf padding key) and the bool [B, S]
    key validity, when the mask is exactly causal ∧ key-padding.  Anything else raises ValueError.

    One pass of rtkv_mask_key_padding over the mask (no [B, S, S] temporaries) and one host sync: key
    validity from the last query row (which sees every unpadded key), every entry checked against it."""
    import ctypes
    from . import _lib as L
    if attention_mask.dim() != 4 or attention_mask.shape[1] != 1 or attention_mask.shape[0] not in (1, B) \
            or attention_mask.shape[2] < S or attention_mask.shape[3] < S:
        raise ValueError(f"attention_mask must be [B, 1, S, S] (got {tuple(attention_mask.shape)})")
    m = attention_mask
    if m.dtype not in L.TORCH_DTYPE_CODE:
        raise ValueError("attention_mask must be the model's additive float32/float16/bfloat16 mask")
    L.require_device(m)
    Bm = m.shape[0]
    # finfo.min / 2 as the comparison `m <= finfo.min / 2` sees it: rounded to the mask's dtype
    thr = float(torch.tensor(torch.finfo(m.dtype).min / 2, dtype=m.dtype).float())
    valid = torch.empty(Bm, S, dtype=torch.uint8, device=m.device)
    counts = torch.zeros(2, dtype=torch.int64, device=m.device)
    L.check(L.lib().rtkv_mask_key_padding(m.data_ptr(), L.TORCH_DTYPE_CODE[m.dtype], Bm, S, m.stride(0), m.stride(2),
                                          m.stride(3), ctypes.c_float(thr), valid.data_ptr(), S, counts.data_ptr(),
                                          L.stream_ptr(m.device)), "rtkv_mask_key_padding")
    bad, padded = (int(x) for x in counts.tolist())  # the one host sync
    if bad:
        raise ValueError("attention_mask is not a causal mask with key padding: every entry must be 0 or "
                         "<= finfo.min/2, and 0 exactly where j <= i and key j is unpadded "
                         f"({bad} entries are not); unsupported by the fused importance mode")
    if padded == 0:
        return None, None
    valid_key = valid.bool().expand(B, S).contiguous()
    bias = torch.zeros(B, S, dtype=torch.float32, device=m.device).masked_fill_(~valid_key, float("-inf"))
    return bias, valid_key
