"""Extension "rtkv-gq/1": per-channel outlier detection + per-head group-wise 2/4/8-bit pack of a layer's
kept K/V rows (include/rtkv.h rtkv_gq_*; kernels in csrc/outlier.hip).

NO REFERENCE COUNTERPART.  The reference quantizes each kept token with ONE (scale, zero_point) over all
H·D channels (src/compression/dynamic_quantization.py:181-194), so a few large-magnitude key channels set
the step of every channel of the row.  BASELINE.json's north_star asks for per-channel outlier detection
and a group-wise pack; this module provides it as an OPT-IN mode (``RealTimePrefillCompressor(config,
group_quant=GroupQuantConfig())``): the reference's K'/V' return values are unchanged, and the layer's
``info["group_quant"]`` additionally holds a :class:`GroupQuantKVCache` — the same kept rows and class
widths, with one (scale, zero_point) per head over the head's non-outlier channels and the layer's outlier
channels (chosen by per-row votes) kept exactly.  Parity is UNPINNED (there is no reference output to pin
it to): oracle/rtkv_oracle.c ``rtkvo_gq_*`` defines the mode and the kernels match it byte for byte
(tests/test_gpu_gq.py).
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass
from typing import Optional

import torch

from . import _lib as L

GQ_D = 128  # head_dim: one group per head


class GqParams(ctypes.Structure):
    _fields_ = [("n_outlier", L.c_i32), ("n_vote", L.c_i32), ("vote_stride", L.c_i32), ("min_votes_pm", L.c_i32)]


@dataclass
class GroupQuantConfig:
    """n_outlier: outlier channels per head and tensor (0..16); n_vote: channels each sampled row votes for
    per head (its n_vote largest |x|); vote_stride: every vote_stride-th kept row votes; min_votes_pm: votes
    a channel needs, per mille of the sampled rows (a channel that is only occasionally large stays in the
    group)."""
    n_outlier: int = 4
    n_vote: int = 4
    vote_stride: int = 4
    min_votes_pm: int = 250

    def params(self) -> GqParams:
        return GqParams(int(self.n_outlier), int(self.n_vote), int(self.vote_stride), int(self.min_votes_pm))

    def min_votes(self, rows: int) -> int:
        """The vote threshold for a layer of `rows` kept rows (as the select kernel computes it)."""
        nsamp = -(-rows // self.vote_stride)
        return max(1, -(-nsamp * self.min_votes_pm // 1000))


def gq_kv_desc(K: torch.Tensor, V: torch.Tensor) -> L.KVDesc:
    """[1, S, H·128] K/V rows (unit feature stride) as H heads of 128 channels."""
    if K.shape != V.shape or K.dtype != V.dtype or K.stride() != V.stride() or K.dim() != 3 or K.stride(-1) != 1:
        raise ValueError("gq: K and V must be [1, S, H*128] with identical strides and unit feature stride")
    B, S, F = K.shape
    if B != 1 or F % GQ_D:
        raise ValueError(f"gq: one batch row of H*128 features (got {tuple(K.shape)})")
    d = L.KVDesc()
    d.k_dev, d.v_dev = K.data_ptr(), V.data_ptr()
    d.dtype = L.dtype_code(K)
    d.B, d.S, d.H, d.D = 1, S, F // GQ_D, GQ_D
    d.stride_b, d.stride_s, d.stride_h = K.stride(0), K.stride(1), GQ_D
    return d


class GroupQuantKVCache:
    """One layer's kept K/V rows in the rtkv-gq/1 format, on the device.

    codes_{k,v}: the codes at the per-token layout's row slots (row_offset, F·w/8 bytes per row); meta
    [rows, 2, H, 2] = {scale, zero_point} per (row, tensor, head) and raw [rows, 2, H, n_outlier] = the
    outlier channels' values, both in the K/V dtype; outlier_idx [2, H, n_outlier] = the layer's outlier
    channels (channel within the head, -1 unused).  kept_index / labels / row_offset / stats are the
    layer's per-token outputs (the rows and their classes)."""

    def __init__(self, K, V, kept_index, labels, row_offset, stats, rows: int, codes_bytes: int, bits, cfg):
        self.cfg = cfg
        self.dtype, self.device = K.dtype, K.device
        self.S, self.F = K.shape[1], K.shape[2]
        self.H = self.F // GQ_D
        self.rows = int(rows)
        self.bits = tuple(int(b) for b in bits)
        self.kept_index, self.labels, self.row_offset, self.stats = kept_index, labels, row_offset, stats
        self._kd = gq_kv_desc(K, V)  # shapes only after packing (the pointers are not read again)
        cap = max(self.rows, 1)
        n = max(int(codes_bytes), 1)
        self.codes_k = torch.empty(n, dtype=torch.uint8, device=self.device)
        self.codes_v = torch.empty(n, dtype=torch.uint8, device=self.device)
        store = torch.float32 if self.dtype == torch.float32 else torch.int16
        self.meta = torch.empty(cap, 2, self.H, 2, dtype=store, device=self.device)
        self.raw = torch.empty(cap, 2, self.H, max(int(cfg.n_outlier), 1), dtype=store, device=self.device)
        self.outlier_idx = torch.full((2, self.H, max(int(cfg.n_outlier), 1)), -1, dtype=torch.int16, device=self.device)
        self._p = cfg.params()
        self._b3 = (ctypes.c_int32 * 3)(*self.bits)

    _ready = None  # set when the cache was produced on a side stream (gq_compress(stream=...))

    def wait(self):
        """Make the current stream wait for the side stream that produced the cache (no-op otherwise); its
        tensors are then also recorded on the current stream, so the allocator keeps them until the
        current stream's work on them is done."""
        if self._ready is not None:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(self._ready)
            for t in (self.codes_k, self.codes_v, self.meta, self.raw, self.outlier_idx, self.kept_index,
                      self.labels, self.row_offset, self.stats):
                t.record_stream(cur)
            self._ready = None
        return self

    def _common(self):
        return (ctypes.byref(self._kd), self.kept_index.data_ptr(), self.labels.data_ptr(), self.stats.data_ptr(),
                self._b3, ctypes.byref(self._p), self.outlier_idx.data_ptr(), self.row_offset.data_ptr())

    def nbytes(self) -> int:
        """Bytes of the packed layer: codes + meta + raw values + the outlier channel lists."""
        e = 4 if self.dtype == torch.float32 else 2
        used = self.row_offset_end()
        return 2 * used + self.rows * 2 * self.H * (2 + self.cfg.n_outlier) * e + self.outlier_idx.numel() * 2

    def row_offset_end(self) -> int:
        return self.codes_k.numel()

    def dequantize(self):
        """(K', V') [1, rows, F] decoded from the format (rtkv_gq_unpack)."""
        self.wait()
        outs = []
        for which, codes in ((0, self.codes_k), (1, self.codes_v)):
            out = torch.empty(1, self.rows, self.F, dtype=self.dtype, device=self.device)
            if self.rows:
                kd, ki, lb, st, b3, p, oi, ro = self._common()
                L.check(L.lib().rtkv_gq_unpack(kd, ki, lb, st, b3, p, oi, ro, codes.data_ptr(), codes.numel(),
                                               self.meta.data_ptr(), self.raw.data_ptr(), self.rows, which,
                                               out.data_ptr(), L.stream_ptr(self.device)), "rtkv_gq_unpack")
            outs.append(out)
        return outs[0], outs[1]

    def attend(self, q: torch.Tensor, scale: Optional[float] = None) -> torch.Tensor:
        """Decode attention of one new token q [1, Hq, 128] (K/V dtype) over the layer, from the codes
        (rtkv_gq_decode_attention): out [1, Hq, 128] fp32."""
        if q.dim() != 3 or q.shape[0] != 1 or q.shape[2] != GQ_D or q.dtype != self.dtype:
            raise ValueError("gq attend: q must be [1, Hq, 128] in the K/V dtype")
        self.wait()
        q = q.contiguous()
        Hq = q.shape[1]
        out = torch.empty(1, Hq, GQ_D, dtype=torch.float32, device=self.device)
        ws = torch.empty(int(L.lib().rtkv_gq_decode_workspace_size(Hq, self.H)), dtype=torch.uint8, device=self.device)
        kd, ki, lb, st, b3, p, oi, ro = self._common()
        s = float(scale) if scale is not None else 1.0 / math.sqrt(GQ_D)
        L.check(L.lib().rtkv_gq_decode_attention(kd, ki, lb, st, b3, p, oi, ro, self.codes_k.data_ptr(),
                                                 self.codes_v.data_ptr(), self.codes_k.numel(), self.meta.data_ptr(),
                                                 self.raw.data_ptr(), max(self.rows, 1), q.data_ptr(), Hq, s,
                                                 out.data_ptr(), ws.data_ptr(), ws.numel(), L.stream_ptr(self.device)),
                "rtkv_gq_decode_attention")
        return out


def gq_compress(K: torch.Tensor, V: torch.Tensor, kept_index: torch.Tensor, labels: torch.Tensor,
                row_offset: torch.Tensor, stats: torch.Tensor, rows: int, codes_bytes: int, bits,
                cfg: Optional[GroupQuantConfig] = None,
                stream: Optional[torch.cuda.Stream] = None) -> GroupQuantKVCache:
    """Outlier channels (rtkv_gq_outlier_channels) and the pack (rtkv_gq_pack) of a compressed layer's kept
    rows, stream-ordered after the layer: K, V [1, S, H·128] (the layer's inputs), kept_index / labels /
    row_offset / stats its per-token outputs (LayerBuffers), rows = S' and codes_bytes = the layer's packed
    bytes per tensor (its published statistics).

    stream: run the launches on this side stream instead (after everything enqueued on the current stream
    so far), so the extension overlaps what the caller enqueues next — the next layer's selection leaves
    most CUs idle for ~20 us.  The inputs are recorded on the side stream (the allocator keeps them until
    it is done); the cache's consumers (dequantize, attend) wait for it, direct reads of its tensors need
    cache.wait() (or a device sync) first."""
    cfg = cfg or GroupQuantConfig()
    L.require_device(K, V)
    if stream is not None:
        stream.wait_stream(torch.cuda.current_stream(K.device))
        for t in (K, V, kept_index, labels, row_offset, stats):
            t.record_stream(stream)
        with torch.cuda.stream(stream):
            c = gq_compress(K, V, kept_index, labels, row_offset, stats, rows, codes_bytes, bits, cfg)
            c._ready = torch.cuda.Event()
            c._ready.record(stream)
        return c
    c = GroupQuantKVCache(K, V, kept_index, labels, row_offset, stats, rows, codes_bytes, bits, cfg)
    if c.rows == 0:
        return c
    st = L.stream_ptr(K.device)
    kd, ki, lb, sp, b3, p, oi, ro = c._common()
    if cfg.n_outlier > 0:
        ws = torch.empty(int(L.lib().rtkv_gq_workspace_size(c.H, GQ_D)), dtype=torch.uint8, device=K.device)
        L.check(L.lib().rtkv_gq_outlier_channels(kd, ki, lb, sp, p, c.rows, oi, ws.data_ptr(), ws.numel(), st),
                "rtkv_gq_outlier_channels")
        c._votes = ws  # (kept until the stream has used it)
    L.check(L.lib().rtkv_gq_pack(kd, ki, lb, sp, b3, p, oi, ro, c.codes_k.data_ptr(), c.codes_v.data_ptr(),
                                 c.codes_k.numel(), c.meta.data_ptr(), c.raw.data_ptr(), c.rows, st), "rtkv_gq_pack")
    return c
