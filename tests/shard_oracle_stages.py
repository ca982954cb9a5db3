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


class OracleShardStages:
    def aggregate(self, W, P, row0, S_total, A_out):
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
