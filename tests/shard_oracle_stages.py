"""TEST INFRASTRUCTURE: oracle-backed stand-ins for rtkv.sharded.HipShardStages.

The CPU suite has no GPU, so the multi-process (gloo) tests of the sequence-sharded orchestration
(rtkv/sharded.py: partitioning, the all-gather of A, rank bounds, the end-of-prefill exchange) run
with these stages, which compute each stage with the C oracle (oracle/rtkv_oracle.c) on CPU tensors
and write the same buffers, in the same layout, as the HIP kernels.  The product path never uses
them: HipShardStages is the default and needs librtkv.so on a ROCm device.
"""
from __future__ import annotations

import numpy as np
import torch

import rtkv_oracle as orc

_CODE = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}


def storage(t: torch.Tensor) -> np.ndarray:
    t = t.detach().contiguous().cpu()
    return t.numpy() if t.dtype == torch.float32 else t.view(torch.int16).numpy().view(np.uint16)


def _put(dst: torch.Tensor, arr: np.ndarray):
    if dst.dtype == torch.float32:
        dst.copy_(torch.from_numpy(np.ascontiguousarray(arr, np.float32)))
    else:
        dst.view(torch.int16).copy_(torch.from_numpy(np.ascontiguousarray(arr, np.uint16).view(np.int16)))


def qk_mass(Q: np.ndarray, K_prompt: np.ndarray, lse: np.ndarray, P: int, row0: int, causal: bool = True):
    """Fused-mode A (token_importance.py:21-47 fed by the softmax of modified_llama.py:88-94, restricted
    to the prompt columns): A[b,i] = (1/H) Σ_h Σ_{p<P, p<=row0+i} exp(q·k/√d − lse), in float64 per row
    (each element from its own dot products, so a row's value does not depend on the rows around it),
    rounded to fp32.  Q [B,H,S,D] float32, K_prompt [B,P',Hkv*D] float32 (P' >= P), lse [B,H,S]."""
    B, H, S, D = Q.shape
    Hkv = K_prompt.shape[2] // D
    k = K_prompt[:, :P].astype(np.float64).reshape(B, P, Hkv, D)
    acc = np.zeros((B, S), np.float64)
    rows = row0 + np.arange(S)
    for b in range(B):
        for h in range(H):
            kh = k[b, :, h // (H // Hkv)]                                   # [P, D]
            x = (Q[b, h].astype(np.float64)[:, None, :] * kh[None]).sum(-1) / np.sqrt(D)   # [S, P]
            w = np.exp(x - lse[b, h].astype(np.float64)[:, None])
            if causal:
                w = np.where(np.arange(P)[None, :] <= rows[:, None], w, 0.0)
            acc[b] += w.sum(-1)
    return (acc / H).astype(np.float32)


class OracleShardStages:
    def aggregate_qk(self, Q, K_prompt, lse, P, row0, causal, A_out):
        A_out.copy_(torch.from_numpy(qk_mass(Q.float().numpy(), K_prompt.float().numpy(), lse.float().numpy(), P,
                                             row0, causal)))

    def aggregate(self, W, P, row0, S_total, A_out, params=None, bufs=None):
        A_out.copy_(torch.from_numpy(orc.attention_aggregation(storage(W), _CODE[W.dtype], P)))

    def finalize(self, A, a_dtype, params, bufs):
        g = bufs.g
        bits = tuple(params.bits)
        A = A.cpu().numpy()
        B, S = A.shape
        scores = orc.importance_scores(A, a_dtype, params.prompt_len, params.alpha, params.beta, params.gamma,
                                       params.layer_weight)
        labels, _ = orc.assign_precision(scores, params.theta_h, params.theta_m)
        mask, kept, _, _ = orc.select(scores, labels, bits, params.propagation_ratio)
        kv_dt = _CODE[bufs.dtype]
        widths = np.array([orc.field_width(kv_dt, b) for b in bits])
        row_bytes = (bufs.F * widths + 7) // 8
        kept_index = np.full((B, S), -1, np.int32)
        row_offset = np.zeros((B, S), np.int64)
        base = 0
        bufs.packed_bytes = []
        for b in range(B):
            idx = np.nonzero(mask[b])[0]
            kept_index[b, :idx.size] = idx
            rb = row_bytes[labels[b, idx]]
            row_offset[b, :idx.size] = base + np.concatenate([[0], np.cumsum(rb)[:-1]]).astype(np.int64)
            row_offset[b, idx.size:] = base + int(rb.sum())  # padding rows: the row's end offset (as K2)
            bufs.packed_bytes.append(int(rb.sum()))
            base += int(rb.sum())
        bufs.kept = kept.astype(np.int64)
        g.scores.copy_(torch.from_numpy(scores))
        g.labels.copy_(torch.from_numpy(labels))
        g.mask.copy_(torch.from_numpy(mask))
        g.kept_index.copy_(torch.from_numpy(kept_index))
        if g.row_offset is not None:
            g.row_offset.copy_(torch.from_numpy(row_offset))

    def ranges(self, bufs, world):
        g = bufs.g
        ki, ro = g.kept_index.numpy(), g.row_offset.numpy()
        out = np.zeros((bufs.B, world + 1, 2), np.int64)
        base = 0
        for b in range(bufs.B):
            k = int(bufs.kept[b])
            for j in range(world + 1):
                lo = k if j == world else int(np.searchsorted(ki[b, :k], j * bufs.S_local, side="left"))
                out[b, j] = (lo, ro[b, lo] if lo < k else base + bufs.packed_bytes[b])
            base += bufs.packed_bytes[b]
        bufs.ranges.copy_(torch.from_numpy(out))

    def quantize(self, K, V, layout, row0, rank, world, params, bufs):
        assert layout == "bsf"
        g = bufs.g
        dt = _CODE[K.dtype]
        bits = tuple(params.bits)
        Kn, Vn = storage(K), storage(V)
        labels, ki, ro = g.labels.numpy(), g.kept_index.numpy(), g.row_offset.numpy()
        rg = bufs.ranges.numpy()
        sz = g.scale_zp.numpy()
        n = int(bufs.kept.max())
        for b in range(bufs.B):
            sz[b, int(bufs.kept[b]):n] = 0.0  # padding rows: zero scale/zp on every rank, as the HIP kernel
            r_lo, r_hi = int(rg[b, rank, 0]), int(rg[b, rank + 1, 0])
            for r in range(r_lo, r_hi):
                i = int(ki[b, r])
                bt = bits[labels[b, i]]
                w = orc.field_width(dt, bt)
                for which, (src, pk, loc) in enumerate(((Kn, g.packed_k, bufs.k_local), (Vn, g.packed_v, bufs.v_local))):
                    row = src[b, i - row0]
                    scale, zp = orc.quant_params(row, dt, bt)
                    codes, deq = orc.fake_quant(row, dt, bt, scale, zp)
                    packed = orc.pack_codes(codes, w)
                    pk[int(ro[b, r]): int(ro[b, r]) + packed.size] = torch.from_numpy(packed)
                    sz[b, r, 2 * which: 2 * which + 2] = (scale, zp)
                    _put(loc[b, r - r_lo], deq)


def single_process_from_A(K, V, dt: int, A: np.ndarray, params, bits, ratio: float) -> dict:
    """The single-process outputs of one layer given its aggregation A (fp32, the fused mode): scores,
    classes and selection by the oracle, every kept row quantized and packed by the oracle — the same
    dict keys as rtkv_oracle.compress_layer (storage arrays)."""
    B, S, F = K.shape
    scores = orc.importance_scores(A, 0, params.prompt_len, params.alpha, params.beta, params.gamma,
                                   params.layer_weight)
    labels, _ = orc.assign_precision(scores, params.theta_h, params.theta_m)
    mask, kept, _, _ = orc.select(scores, labels, tuple(bits), ratio)
    widths = [orc.field_width(dt, b) for b in bits]
    rows = [np.nonzero(mask[b])[0] for b in range(B)]
    n = max(r.size for r in rows)
    out_dt = np.float32 if dt == 0 else np.uint16
    k_out = np.zeros((B, n, F), out_dt)
    v_out = np.zeros((B, n, F), out_dt)
    kept_index = np.zeros((B, n), np.int32)
    row_offset = np.zeros((B, n), np.int64)
    scale_zp = np.zeros((B, n, 4), np.float32)
    pk, pv = [], []
    base = 0
    for b in range(B):
        for r, i in enumerate(rows[b]):
            bt = bits[labels[b, i]]
            w = widths[labels[b, i]]
            kept_index[b, r] = i
            row_offset[b, r] = base
            for which, (src, dst, packs) in enumerate(((K, k_out, pk), (V, v_out, pv))):
                scale, zp = orc.quant_params(src[b, i], dt, bt)
                codes, deq = orc.fake_quant(src[b, i], dt, bt, scale, zp)
                packs.append(orc.pack_codes(codes, w))
                dst[b, r] = deq
                scale_zp[b, r, 2 * which: 2 * which + 2] = (scale, zp)
            base += packs[-1].size
        row_offset[b, rows[b].size:] = base
    return {"max_kept": n, "kept_index": kept_index, "mask": mask, "row_offset": row_offset, "scale_zp": scale_zp,
            "packed_k": np.concatenate(pk) if pk else np.zeros(0, np.uint8),
            "packed_v": np.concatenate(pv) if pv else np.zeros(0, np.uint8), "k_out": k_out, "v_out": v_out}
