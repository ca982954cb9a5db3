"""A random-init Llama-2-7B-shaped decoder for the sync'd prefill wall-time leg of bench.py (SURVEY
§8d, BASELINE.md §3: TTFT as `src/evaluation/benchmark runner.py:202-212` measures it — one forward
pass with use_cache, torch.cuda.synchronize() after it).

Not part of the product: the model around the compression path (embedding, RMSNorm, projections,
RoPE, SwiGLU MLP, LM head) is plain PyTorch with weights ~ N(0, 0.02) (HF's initializer_range), made
directly on the device.  Three attention variants per layer, all with the cache the layer hands on:

* ``none``:  SDPA over the full K/V (uncompressed cache) — the model without compression;
* ``fused``: rtkv.CompressedPrefillAttention (row LSE + fused-mode compression on the GPU, then the
  reference's attention over K'/V'; no [B,H,S,S] tensor) — this repo's model-side path;
* ``eager``: the reference layer's own structure (modified_llama.py:88-142): the materialised
  softmax(QKᵀ/√d + mask) in fp32, cast to the model dtype, handed to
  RealTimePrefillCompressor.compress_layer_kv_cache (the W path), then the attention recomputed over
  K' with the first S' mask columns.
"""
from __future__ import annotations

import math
import time
from typing import Dict, List

import torch
import torch.nn.functional as Fn

LLAMA2_7B = dict(vocab=32000, hidden=4096, layers=32, heads=32, kv_heads=32, inter=11008, eps=1e-5, theta=10000.0)


class RandomLlama:
    def __init__(self, device, dtype=torch.float16, seed=0, **shape):
        c = dict(LLAMA2_7B, **shape)
        self.c = c
        self.dtype = dtype
        g = torch.Generator(device=device).manual_seed(seed)
        H, D = c["heads"], c["hidden"] // c["heads"]
        self.H, self.Hkv, self.D = H, c["kv_heads"], D

        def w(*s):
            return (torch.randn(*s, device=device, generator=g, dtype=torch.float32) * 0.02).to(dtype)

        self.embed = w(c["vocab"], c["hidden"])
        self.layers = []
        for _ in range(c["layers"]):
            self.layers.append(dict(
                ln1=torch.ones(c["hidden"], device=device, dtype=dtype),
                qkv=w((H + 2 * self.Hkv) * D, c["hidden"]),   # q_proj, k_proj, v_proj stacked
                o=w(c["hidden"], H * D),
                ln2=torch.ones(c["hidden"], device=device, dtype=dtype),
                gu=w(2 * c["inter"], c["hidden"]),             # gate_proj, up_proj stacked
                down=w(c["hidden"], c["inter"])))
        self.norm = torch.ones(c["hidden"], device=device, dtype=dtype)
        self.lm_head = w(c["vocab"], c["hidden"])
        inv = 1.0 / (c["theta"] ** (torch.arange(0, D, 2, device=device, dtype=torch.float32) / D))
        self.inv_freq = inv

    def rms(self, x, w):
        v = x.float().pow(2).mean(-1, keepdim=True)
        return (x.float() * torch.rsqrt(v + self.c["eps"])).to(self.dtype) * w

    def rope(self, S, device):
        t = torch.arange(S, device=device, dtype=torch.float32)
        f = torch.outer(t, self.inv_freq)
        emb = torch.cat([f, f], -1)
        return emb.cos().to(self.dtype), emb.sin().to(self.dtype)

    @staticmethod
    def rot(x, cos, sin):
        h = x.shape[-1] // 2
        return x * cos + torch.cat([-x[..., h:], x[..., :h]], -1) * sin

    @torch.no_grad()
    def prefill(self, ids: torch.Tensor, mode: str, attn_layers=None, compressor=None) -> Dict:
        """One forward pass over ids [B, S] with the cache built; returns logits and the per-layer cache."""
        B, S = ids.shape
        H, Hkv, D = self.H, self.Hkv, self.D
        cos, sin = self.rope(S, ids.device)
        h = self.embed[ids]
        cache: List = []
        kept = 0
        for li, L in enumerate(self.layers):
            x = self.rms(h, L["ln1"])
            qkv = x @ L["qkv"].t()
            q = qkv[..., : H * D].view(B, S, H, D).transpose(1, 2)
            k = qkv[..., H * D:(H + Hkv) * D].view(B, S, Hkv, D).transpose(1, 2)
            v = qkv[..., (H + Hkv) * D:].view(B, S, Hkv, D).transpose(1, 2)
            q, k = self.rot(q, cos, sin), self.rot(k, cos, sin)
            if mode == "none":
                o = Fn.scaled_dot_product_attention(q, k, v.contiguous(), is_causal=True, enable_gqa=Hkv != H)
                cache.append((k, v))
                kept += S
            elif mode == "fused":
                o, kv, _ = attn_layers[li](q.contiguous(), k.contiguous(), v.contiguous(), ids)
                cache.append(kv)
                kept += kv[0].shape[2]
            elif mode == "eager":
                o, kv = self._eager_layer(q, k, v, ids, li, compressor)
                cache.append(kv)
                kept += kv[0].shape[2]
            else:
                raise ValueError(mode)
            h = h + o.transpose(1, 2).reshape(B, S, H * D) @ L["o"].t()
            x = self.rms(h, L["ln2"])
            gu = x @ L["gu"].t()
            inter = self.c["inter"]
            h = h + (Fn.silu(gu[..., :inter]) * gu[..., inter:]) @ L["down"].t()
        logits = self.rms(h, self.norm) @ self.lm_head.t()
        return {"logits": logits, "cache": cache, "kept_rows": kept}

    def _eager_layer(self, q, k, v, ids, li, compressor):
        """modified_llama.py:88-142 literally (GQA by head repetition as the model's repeat_kv)."""
        B, H, S, D = q.shape
        Hkv = k.shape[1]
        g = H // Hkv
        kr = k.repeat_interleave(g, dim=1) if g > 1 else k
        mask = torch.full((S, S), torch.finfo(self.dtype).min, device=q.device, dtype=self.dtype).triu(1)
        w = torch.matmul(q, kr.transpose(2, 3)) / math.sqrt(D) + mask
        w = torch.softmax(w, dim=-1, dtype=torch.float32).to(self.dtype)
        kf = k.transpose(1, 2).reshape(B, S, Hkv * D).contiguous()
        vf = v.transpose(1, 2).reshape(B, S, Hkv * D).contiguous()
        k2, v2, _ = compressor.compress_layer_kv_cache(kf, vf, w, ids, li)
        del w
        Sp = k2.shape[1]
        ck = k2.view(B, Sp, Hkv, D).transpose(1, 2)
        cv = v2.view(B, Sp, Hkv, D).transpose(1, 2)
        ckr = ck.repeat_interleave(g, dim=1) if g > 1 else ck
        cvr = cv.repeat_interleave(g, dim=1) if g > 1 else cv
        cw = torch.matmul(q, ckr.transpose(2, 3)) / math.sqrt(D) + mask[:, :Sp]
        cw = torch.softmax(cw, dim=-1, dtype=torch.float32).to(self.dtype)
        o = torch.matmul(cw, cvr)
        return o, (ck, cv)


def prefill_leg(device, S=16384, dtype=torch.float16, modes=("none", "fused", "eager"), reps=2, layers=None,
                compression=None) -> Dict:
    """Sync'd prefill wall time (ms) of the random-init 7B-shaped model at S tokens per mode."""
    import rtkv
    from rtkv.model_side import CompressedPrefillAttention
    shape = {} if layers is None else {"layers": layers}
    model = RandomLlama(device, dtype=dtype, **shape)
    c = model.c
    cfg = rtkv.CompressionConfig(num_hidden_layers=c["layers"], **(compression or {}))
    g = torch.Generator(device=device).manual_seed(1)
    ids = torch.randint(0, c["vocab"], (1, S), device=device, generator=g)
    out = {"model": f"random-init Llama-2-7B shape ({c['layers']} layers, {c['heads']}x{model.D}, hidden "
                    f"{c['hidden']}, MLP {c['inter']}, vocab {c['vocab']})", "seq": S,
           "dtype": str(dtype).split(".")[-1], "reps": reps,
           "timing": "torch.cuda.synchronize(); t0; model forward (logits + per-layer cache); "
                     "torch.cuda.synchronize(); t1 — benchmark runner.py:202-212"}
    for mode in modes:
        comp = rtkv.RealTimePrefillCompressor(cfg) if mode != "none" else None
        attn = [CompressedPrefillAttention(comp, c["heads"], c["kv_heads"], model.D, li) for li in range(c["layers"])] \
            if mode == "fused" else None
        try:
            r = model.prefill(ids, mode, attn, comp)  # warm-up (kernel selection, allocator)
            del r
            torch.cuda.synchronize(device)
            ts = []
            for _ in range(reps):
                if comp is not None:
                    comp.reset_compression_state()
                torch.cuda.synchronize(device)
                t0 = time.perf_counter()
                r = model.prefill(ids, mode, attn, comp)
                torch.cuda.synchronize(device)
                ts.append((time.perf_counter() - t0) * 1e3)
                kept = r["kept_rows"]
                del r
            out[mode] = {"ttft_ms": round(min(ts), 2), "ttft_ms_all": [round(t, 2) for t in ts],
                         "kept_rows_all_layers": int(kept),
                         "cache_rows_fraction": round(kept / (S * c["layers"]), 4)}
        except torch.OutOfMemoryError as e:  # the eager variant's [B,H,S,S] softmax at long S
            out[mode] = {"error": f"out of memory: {str(e).splitlines()[0][:160]}"}
        finally:
            torch.cuda.empty_cache()
    if "none" in out and "fused" in out and "ttft_ms" in out["fused"]:
        out["fused_overhead_ms"] = round(out["fused"]["ttft_ms"] - out["none"]["ttft_ms"], 2)
    del model
    torch.cuda.empty_cache()
    return out
