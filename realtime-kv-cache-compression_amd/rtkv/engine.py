"""Device-side driver of one layer's compression (the C ABI's rtkv_compress_layer) with reusable
output buffers.  Everything here is stream-ordered and sync-free except ``LayerResult.stats()``.

This is the layer the reference-mirroring classes (unified_compressor.py etc.) and bench.py use.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from . import _lib as L


def params_from_config(config, layer_idx: int, prompt_len: int, ratio: float, flags: int) -> L.LayerParams:
    """rtkv_layer_params for one layer.  ctypes.c_float performs the same double→float32 rounding
    PyTorch applies to a Python scalar combined with an fp32 tensor."""
    p = L.LayerParams()
    p.alpha = float(config.alpha)
    p.beta = float(config.beta)
    p.gamma = float(config.gamma)
    p.layer_weight = float(config.layer_weights[layer_idx])
    p.theta_h = float(config.theta_h)
    p.theta_m = float(config.theta_m)
    p.bits[0] = int(config.low_precision_bits)
    p.bits[1] = int(config.medium_precision_bits)
    p.bits[2] = int(config.high_precision_bits)
    p.prompt_len = int(prompt_len)
    p.propagation_ratio = float(ratio)
    p.flags = int(flags)
    return p


def prompt_length(seq_len: int) -> int:
    """unified_compressor.py:55"""
    return max(1, min(seq_len // 5, 128))


def attn_desc(W: torch.Tensor) -> L.AttnDesc:
    if W.dim() != 4:
        raise ValueError(f"attention weights must be [B, H, S, cols], got {tuple(W.shape)}")
    if W.stride(-1) != 1:
        raise ValueError("attention weights must have unit stride along the last (key) dimension")
    d = L.AttnDesc()
    d.w_dev = W.data_ptr()
    d.dtype = L.dtype_code(W)
    d.B, d.H, d.S, d.cols = W.shape
    d.stride_b, d.stride_h, d.stride_s = W.stride(0), W.stride(1), W.stride(2)
    return d


def kv_desc(K: torch.Tensor, V: torch.Tensor, layout: str = "bsf", heads: Optional[int] = None) -> L.KVDesc:
    """layout 'bsf': [B, S, F] (the reference's compress_layer_kv_cache input);
    layout 'bhsd': [B, H, S, D] (the model-native layout, no transpose copy)."""
    if K.shape != V.shape or K.dtype != V.dtype or K.stride() != V.stride():
        raise ValueError("key and value states must have identical shape, dtype and strides")
    d = L.KVDesc()
    d.k_dev, d.v_dev = K.data_ptr(), V.data_ptr()
    d.dtype = L.dtype_code(K)
    if layout == "bsf":
        if K.dim() != 3 or K.stride(-1) != 1:
            raise ValueError("bsf layout needs [B, S, F] with unit feature stride")
        B, S, F = K.shape
        d.B, d.S, d.H, d.D = B, S, 1, F
        d.stride_b, d.stride_s, d.stride_h = K.stride(0), K.stride(1), F
    elif layout == "bhsd":
        if K.dim() != 4 or K.stride(-1) != 1:
            raise ValueError("bhsd layout needs [B, H, S, D] with unit head_dim stride")
        B, H, S, D = K.shape
        d.B, d.S, d.H, d.D = B, S, H, D
        d.stride_b, d.stride_s, d.stride_h = K.stride(0), K.stride(2), K.stride(1)
    else:
        raise ValueError(layout)
    return d


def qk_desc(Q: torch.Tensor, K: torch.Tensor, lse: torch.Tensor, scale: Optional[float] = None,
            causal: bool = True, k_layout: str = "bsf", kv_heads: Optional[int] = None, row0: int = 0,
            key_bias: Optional[torch.Tensor] = None) -> L.QKDesc:
    """Fused importance input: Q [B,H,S,D] (model layout, unit d stride), keys whose first P rows are
    the prompt keys — K [B,S,Hkv*D] ('bsf', the reference's compress_layer_kv_cache input) or
    [B,Hkv,S,D] ('bhsd') — and the row log-sum-exp lse [B,H,S] (fp32) of the model's softmax.
    key_bias: optional fp32 [B, S] additive key-padding bias (0 real key, -inf padding key), the
    padding part of the model's attention_mask (modified_llama.py:90-91)."""
    if Q.dim() != 4 or Q.stride(-1) != 1:
        raise ValueError("queries must be [B, H, S, D] with unit head_dim stride")
    B, H, S, D = Q.shape
    if K.dtype != Q.dtype:
        raise ValueError("queries and keys must share a dtype")
    if lse.dtype != torch.float32 or tuple(lse.shape) != (B, H, S) or lse.stride(-1) != 1:
        raise ValueError(f"lse must be float32 [B, H, S] = {(B, H, S)} with unit stride")
    d = L.QKDesc()
    d.q_dev, d.k_dev, d.lse_dev = Q.data_ptr(), K.data_ptr(), lse.data_ptr()
    d.dtype = L.dtype_code(Q)
    d.causal = int(bool(causal))
    d.B, d.H, d.S, d.D = B, H, S, D
    d.q_stride_b, d.q_stride_h, d.q_stride_s = Q.stride(0), Q.stride(1), Q.stride(2)
    if k_layout == "bsf":
        if K.dim() != 3 or K.stride(-1) != 1 or K.shape[2] % D:
            raise ValueError("bsf keys must be [B, S, Hkv*D] with unit stride")
        d.Hkv = K.shape[2] // D
        d.k_stride_b, d.k_stride_h, d.k_stride_s = K.stride(0), D, K.stride(1)
    elif k_layout == "bhsd":
        if K.dim() != 4 or K.stride(-1) != 1 or K.shape[3] != D:
            raise ValueError("bhsd keys must be [B, Hkv, S, D] with unit stride")
        d.Hkv = K.shape[1]
        d.k_stride_b, d.k_stride_h, d.k_stride_s = K.stride(0), K.stride(1), K.stride(2)
    else:
        raise ValueError(k_layout)
    d.lse_stride_b, d.lse_stride_h = lse.stride(0), lse.stride(1)
    d.scale = float(scale) if scale is not None else 1.0 / float(D) ** 0.5
    d.row0 = int(row0)
    if key_bias is not None:
        if key_bias.dtype != torch.float32 or key_bias.dim() != 2 or tuple(key_bias.shape) != (B, S) \
                or key_bias.stride(-1) != 1 or key_bias.device != Q.device:
            raise ValueError(f"key_bias must be float32 [B, S] = {(B, S)} with unit stride on the queries' device")
        if row0 != 0:
            raise ValueError("key_bias is not supported for sequence shards (row0 != 0)")
        d.kbias_dev, d.kbias_stride_b = key_bias.data_ptr(), key_bias.stride(0)
    return d


def check_flags(flags: int, what: str = "compress_layer"):
    """Raise for the RTKV_FLAG_* bits that make a layer's outputs invalid."""
    if flags & L.FLAG_SPIN_TIMEOUT:
        raise RuntimeError(f"rtkv: {what} failed (RTKV_ERR_TIMEOUT): a cross-workgroup hand-off of the selection "
                           "kernel did not arrive within its poll bound; the layer's outputs are invalid (NaN rows, "
                           "RTKV_FLAG_SPIN_TIMEOUT)")
    if flags & L.FLAG_OUTPUT_OVERFLOW:
        raise RuntimeError(f"rtkv: {what} failed: the output buffers are smaller than the layer's published sizes; "
                           "nothing was written (RTKV_FLAG_OUTPUT_OVERFLOW)")


@dataclass
class LayerStats:
    max_kept: int
    total_packed_bytes: int
    score_sum: float
    score_m2: float
    score_min: float
    score_max: float
    error_flags: int
    batch: list  # per batch row dicts


def decode_stats(raw: bytes, B: int) -> LayerStats:
    h = L.LayerStatsHeader.from_buffer_copy(raw[: ctypes.sizeof(L.LayerStatsHeader)])
    rows = []
    off = ctypes.sizeof(L.LayerStatsHeader)
    for _ in range(B):
        s = L.BatchStats.from_buffer_copy(raw[off: off + ctypes.sizeof(L.BatchStats)])
        off += ctypes.sizeof(L.BatchStats)
        rows.append(dict(class_count=list(s.class_count), kept=s.kept, kept_class=list(s.kept_class),
                         cost_units=s.cost_units, packed_bytes=s.packed_bytes, fallback=bool(s.fallback),
                         kept_score_sum=s.kept_score_sum))
    return LayerStats(h.max_kept, h.total_packed_bytes, h.score_sum, h.score_m2, h.score_min, h.score_max,
                      h.error_flags, rows)


def _early_to_stats(e: L.EarlyStats) -> LayerStats:
    """Statistics published early by the device (score_m2 / kept_score_sum are not final there; B = 1, complete,
    so kept = max_kept and packed_bytes = total_packed_bytes)."""
    row = dict(class_count=list(e.class_count), kept=e.max_kept, kept_class=list(e.kept_class), cost_units=e.cost_units,
               packed_bytes=e.total_packed_bytes, fallback=False, kept_score_sum=float("nan"))
    return LayerStats(e.max_kept, e.total_packed_bytes, e.score_sum, float("nan"), e.score_min, e.score_max,
                      e.error_flags, [row])


class EarlyStatsBuffer:
    """Host-mapped rtkv_early_stats (rtkv_host_alloc) that the device fills with a layer's final
    counts as soon as K2 has its thresholds, plus the call sequence counter (one per device)."""

    TIMEOUT_US = 20_000_000

    def __init__(self):
        self._lib = L.lib()
        self.ptr = self._lib.rtkv_host_alloc(ctypes.sizeof(L.EarlyStats))
        if not self.ptr:
            raise RuntimeError("rtkv: rtkv_host_alloc failed (pinned host memory for the early statistics)")
        self._view = L.EarlyStats.from_address(self.ptr)  # the pinned block in place (read after the seq word)
        self.seq = 0

    def next_seq(self) -> int:
        self.seq += 1
        return self.seq

    def _read(self) -> L.EarlyStats:
        return L.EarlyStats.from_buffer_copy(self._view)

    def final_flags(self, seq: int) -> Optional[int]:
        """The final RTKV_FLAG_* word K4 published for call `seq` (rtkv_compress_layer_finish), or None
        while that K4 has not started (or a later layer's K4 has overwritten it)."""
        w = ctypes.c_uint64.from_address(ctypes.addressof(self._view) + L.EarlyStats.final_word.offset).value
        if (w >> 16) != (seq & L.FINAL_SEQ_MASK):
            return None
        return int(w & 0xffff)

    def wait_final(self, seq: int, device=None) -> int:
        """The final RTKV_FLAG_* word of call `seq` once its K4 has started and published it
        (rtkv_wait_final); past the timeout the device is synchronised and the mirror re-read."""
        rc = self._lib.rtkv_wait_final(self.ptr, seq, self.TIMEOUT_US)
        if rc == L.ERR_TIMEOUT:
            # a queue slower than the timeout, or a K4 that never published: after a device sync the flags
            # are either in the mirror or (None) read from the statistics block by the caller
            torch.cuda.synchronize(device)
            return self.final_flags(seq)
        L.check(rc, "rtkv_wait_final")
        return int(self._view.final_word & 0xffff)

    def wait(self, seq: int, device=None) -> L.EarlyStats:
        """The statistics of call `seq` once the device has published them.  A queue slower than the
        spin timeout (a long backlog, preemption) is not an error: the device that runs the layer is
        then synchronised and the mirror re-read; only a layer that finished without publishing
        raises."""
        rc = self._lib.rtkv_wait_early(self.ptr, seq, self.TIMEOUT_US)
        if rc == L.ERR_TIMEOUT:
            torch.cuda.synchronize(device)  # also surfaces a device fault, if that is what happened
            e = self._read()
            if e.seq == seq and e.seq_tail == seq:
                rc = 0
        L.check(rc, "rtkv_wait_early")
        return self._read()

    def __del__(self):
        if getattr(self, "ptr", None):
            self._lib.rtkv_host_free(self.ptr)
            self.ptr = None


class Workspace:
    """Caller-owned scratch for the C ABI, grown on demand (one per device).

    Between compress_layer_begin and PendingLayer.finish the workspace belongs to the pending layer
    (K2 leaves the kept rows' classes and the selection scratch there for K4): ``get`` refuses to hand
    it out meanwhile (include/rtkv.h, rtkv_compress_layer_begin)."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.buf = torch.empty(0, dtype=torch.uint8, device=self.device)
        self.pending = None  # the PendingLayer that owns the workspace until its finish()

    def get(self, B: int, S: int, H: Optional[int] = None) -> torch.Tensor:
        """H: query heads of the fused importance mode (room for the head-major K1' scratch)."""
        if self.pending is not None:
            raise RuntimeError("rtkv: the workspace belongs to a layer begun with compress_layer_begin whose "
                               "finish() has not run; finish it (or use another Workspace) first")
        need = int(L.lib().rtkv_workspace_size(B, S) if H is None else L.lib().rtkv_workspace_size_qk(B, H, S))
        if self.buf.numel() < need:
            self.buf = torch.empty(need, dtype=torch.uint8, device=self.device)
        return self.buf


class LayerBuffers:
    """Output buffers of one compressed layer, sized for B batch rows of S tokens (capacity = S).

    Every buffer is a slice of ONE device allocation (the drop-in path creates fresh buffers per
    layer call, as the reference returns fresh tensors; one allocation instead of ten keeps that
    cheap).  Slices are 256-byte aligned.  The kernels need only their addresses (``out_struct``), so
    the tensor views (a few µs of host time each) are made on first access."""

    def __init__(self, B: int, S: int, F: int, dtype: torch.dtype, device, bits, emit_dequant=True, emit_packed=True,
                 outputs: bool = True, row_offsets: bool = False):
        """outputs=False: only the per-token buffers (scores, classes, mask, kept indices, row offsets,
        scale/zero-points, statistics); the caller supplies exactly-sized K'/V' and packed buffers to
        finish() (rtkv_compress_layer_begin / _finish).  row_offsets: the kept rows' code offsets even
        without packed codes (the group-wise extension uses the per-token row slots)."""
        self.B, self.S, self.F, self.dtype = B, S, F, dtype
        self.emit_dequant, self.emit_packed = emit_dequant, emit_packed
        dev = self.device = torch.device(device)
        esz = dtype.itemsize
        cap = 0
        if emit_packed and outputs:
            b3 = (ctypes.c_int32 * 3)(*bits)
            cap = int(L.lib().rtkv_packed_capacity(B, S, F, L.TORCH_DTYPE_CODE[dtype], b3))
        plan = [("scores", B * S * 4, torch.float32, (B, S)), ("labels", B * S, torch.uint8, (B, S)),
                ("mask", B * S, torch.uint8, (B, S)), ("kept_index", B * S * 4, torch.int32, (B, S)),
                ("stats", L.stats_bytes(B), torch.uint8, (L.stats_bytes(B),))]
        if emit_dequant and outputs:
            plan += [("k_out", B * S * F * esz, dtype, (B * S * F,)), ("v_out", B * S * F * esz, dtype, (B * S * F,))]
        if emit_packed and outputs:
            plan += [("packed_k", max(cap, 1), torch.uint8, (max(cap, 1),)),
                     ("packed_v", max(cap, 1), torch.uint8, (max(cap, 1),))]
        if emit_packed or row_offsets:
            plan += [("row_offset", B * S * 8, torch.int64, (B, S)), ("scale_zp", B * S * 16, torch.float32, (B, S, 4))]
        offs, total = {}, 0
        for name, n, dt, shape in plan:
            offs[name] = (total, n, dt, shape)
            total += (n + 255) // 256 * 256
        self.arena = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
        self._base = self.arena.data_ptr()
        self._offs = offs
        for name in ("k_out", "v_out", "packed_k", "packed_v", "row_offset", "scale_zp"):
            if name not in offs:
                setattr(self, name, None)
        self.packed_capacity = cap if (emit_packed and outputs) else 0

    def __getattr__(self, name):
        """The view of buffer `name`, made (and kept) on first access."""
        offs = self.__dict__.get("_offs")
        if offs is None or name not in offs:
            raise AttributeError(name)
        o, n, dt, shape = offs[name]
        v = self.arena[o:o + n].view(dt).view(shape)
        self.__dict__[name] = v
        return v

    def ptr(self, name: str) -> int:
        """Device address of buffer `name` (0 when absent), without making its view."""
        o = self._offs.get(name)
        return self._base + o[0] if o is not None else 0

    def matches(self, B, S, F, dtype, emit_dequant, emit_packed) -> bool:
        return (self.B, self.S, self.F, self.dtype) == (B, S, F, dtype) and \
            ("k_out" in self._offs) == emit_dequant and ("packed_k" in self._offs) == emit_packed

    def out_struct(self, packed_batch_rows: bool = True) -> L.LayerOut:
        o = L.LayerOut()
        p = self.ptr
        o.k_out_dev, o.v_out_dev = p("k_out"), p("v_out")
        # dequant rows packed back to back at the runtime row count: a contiguous [B, S', F] view
        o.o_stride_b = -1 if packed_batch_rows else self.S * self.F
        o.o_stride_s, o.o_stride_h = self.F, self.F
        o.row_capacity = self.S
        o.scores_dev, o.labels_dev, o.mask_dev = p("scores"), p("labels"), p("mask")
        o.kept_index_dev = p("kept_index")
        o.packed_k_dev, o.packed_v_dev = p("packed_k"), p("packed_v")
        o.packed_capacity = self.packed_capacity
        o.row_offset_dev, o.scale_zp_dev = p("row_offset"), p("scale_zp")
        o.stats_dev = p("stats")
        return o


class LayerResult:
    """Device outputs of one rtkv_compress_layer call; ``stats()`` is the single host sync.

    With early statistics (``early`` set: the call published them), ``stats()`` waits only for the
    device's publication — K2's tail and K4 may still be running — and its score_m2 /
    kept_score_sum are NaN; ``final_stats()`` syncs the stream and reads them all."""

    def __init__(self, bufs: LayerBuffers, B: int, early: Optional[EarlyStatsBuffer] = None, seq: int = 0,
                 stream: Optional[int] = None, record: bool = True):
        self.bufs = bufs
        self.B = B
        self._early, self._seq = early, seq
        self._stats: Optional[LayerStats] = None
        self._final: Optional[LayerStats] = None
        # the layer's completion on the stream it was launched on: final_stats() waits for exactly that,
        # whatever stream is current when it is called (no timing: the layer's time span comes from the
        # kernels' own stamps, device_seconds())
        self.done = torch.cuda.Event()
        if record:
            self._record(stream)

    def _record(self, stream: Optional[int]):
        cur = torch.cuda.current_stream(self.bufs.device)
        self.done.record(cur if stream is None or stream == cur.cuda_stream
                         else torch.cuda.ExternalStream(stream, device=self.bufs.device))

    @staticmethod
    def _checked(st: LayerStats) -> LayerStats:
        check_flags(st.error_flags)
        return st

    def stats(self) -> LayerStats:
        if self._stats is None:
            if self._early is not None:
                e = self._early.wait(self._seq, self.bufs.device)
                if e.complete:
                    self._stats = self._checked(_early_to_stats(e))
                    return self._stats
            self._stats = self.final_stats()
        return self._stats

    def final_stats(self) -> LayerStats:
        return self._checked(self.final_stats_unchecked())

    def final_stats_unchecked(self) -> LayerStats:
        """The final statistics block (a stream sync), error flags included but not raised."""
        if self._final is None:
            self.wait_done()
            self._final = decode_stats(self.bufs.stats.cpu().numpy().tobytes(), self.B)
        return self._final

    def device_seconds(self) -> float:
        """The layer's device time span (rtkv_layer_times: the first K1 block's start to the last K4
        workgroup's end on the GPU's real-time counter), after a wait for the layer; NaN when K4 did not
        run (or the call did not stamp it)."""
        if not getattr(self, "finished", True):  # a pending layer whose K4 was never enqueued
            return float("nan")
        self.wait_done()  # (a statistics block read before K4 — the synchronised path — has no end yet)
        t = self.bufs.stats[-L.TIMES_BYTES:].cpu().numpy().view(np.uint64)
        end, begin = int(t[:-1:16].max()), int(t[-1])
        khz = L.wall_clock_khz(self.bufs.device)
        if end == 0 or end < begin or khz <= 0:
            return float("nan")
        return (end - begin) / (khz * 1e3)

    def wait_done(self):
        """Wait for the layer's kernels (its completion event: the layer's stream, not whichever stream
        is current here)."""
        self.done.synchronize()

    def kv(self):
        """Dequantized (K', V') as contiguous [B, S'_max, F] views (reference return value)."""
        st = self.stats()
        n = self.B * st.max_kept * self.bufs.F
        shape = (self.B, st.max_kept, self.bufs.F)
        return self.bufs.k_out[:n].view(shape), self.bufs.v_out[:n].view(shape)


def compress_layer_qk(K, V, Q, lse, params: L.LayerParams, bufs: LayerBuffers, workspace: Workspace,
                      layout: str = "bsf", causal: bool = True, scale: Optional[float] = None,
                      stream: Optional[int] = None, early: Optional[EarlyStatsBuffer] = None,
                      key_bias: Optional[torch.Tensor] = None) -> LayerResult:
    """compress_layer in the fused importance mode: K1' computes A from Q, the prompt keys (the first
    P rows of K) and the row LSE on MFMA; K2 and K4 are unchanged."""
    L.require_device(K, V, Q, lse)
    kd = kv_desc(K, V, layout)
    qd = qk_desc(Q, K, lse, scale=scale, causal=causal, k_layout=layout, key_bias=key_bias)
    if qd.B != kd.B or qd.S != kd.S:
        raise ValueError(f"queries {tuple(Q.shape)} do not match key states {tuple(K.shape)}")
    ws = workspace.get(kd.B, kd.S, H=qd.H)
    out = bufs.out_struct()
    out.o_stride_h = kd.D
    st = L.stream_ptr(K.device) if stream is None else stream
    if early is not None:
        seq, pub = early.next_seq(), ctypes.c_int32(0)
        rc = L.lib().rtkv_compress_layer_qk_early(ctypes.byref(kd), ctypes.byref(qd), ctypes.byref(params),
                                                  ctypes.byref(out), ws.data_ptr(), ws.numel(), st, early.ptr, seq,
                                                  ctypes.byref(pub))
        L.check(rc, "rtkv_compress_layer_qk_early")
        return LayerResult(bufs, kd.B, early if pub.value else None, seq, stream=st)
    rc = L.lib().rtkv_compress_layer_qk(ctypes.byref(kd), ctypes.byref(qd), ctypes.byref(params), ctypes.byref(out),
                                        ws.data_ptr(), ws.numel(), st)
    L.check(rc, "rtkv_compress_layer_qk")
    return LayerResult(bufs, kd.B, stream=st)


def importance_qk_lse(Q, K, lse, prompt_len: int, causal: bool = True, scale: Optional[float] = None,
                      k_layout: str = "bsf", key_bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """A [B, S] (fp32) of the fused importance mode alone (rtkv_importance_qk_lse)."""
    L.require_device(Q, K, lse)
    qd = qk_desc(Q, K, lse, scale=scale, causal=causal, k_layout=k_layout, key_bias=key_bias)
    A = torch.empty(qd.B, qd.S, dtype=torch.float32, device=Q.device)
    scratch = torch.empty(int(L.lib().rtkv_qk_scratch_size(qd.B, qd.H, qd.S)), dtype=torch.uint8, device=Q.device)
    L.check(L.lib().rtkv_importance_qk_lse_ws(ctypes.byref(qd), int(prompt_len), A.data_ptr(), scratch.data_ptr(),
                                              scratch.numel(), L.stream_ptr(Q.device)), "rtkv_importance_qk_lse_ws")
    return A


def attention_lse(Q, K, causal: bool = True, scale: Optional[float] = None, k_layout: str = "bhsd",
                  key_bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Row log-sum-exp [B, H, S] (fp32) of softmax(Q·Kᵀ·scale + causal mask + key_bias) (rtkv_attention_lse):
    the lse the fused importance mode consumes, without the [B, H, S, S] matrix.  A row that sees no
    key (a padding row) gets -inf."""
    L.require_device(Q, K)
    B, H, S, _ = Q.shape
    lse = torch.empty(B, H, S, dtype=torch.float32, device=Q.device)
    qd = qk_desc(Q, K, lse, scale=scale, causal=causal, k_layout=k_layout, key_bias=key_bias)
    L.check(L.lib().rtkv_attention_lse(ctypes.byref(qd), lse.data_ptr(), L.stream_ptr(Q.device)), "rtkv_attention_lse")
    return lse


def compress_layer(K, V, W, params: L.LayerParams, bufs: LayerBuffers, workspace: Workspace,
                   layout: str = "bsf", stream: Optional[int] = None,
                   early: Optional[EarlyStatsBuffer] = None) -> LayerResult:
    """Enqueue aggregation → scores/labels/selection → quantize+pack+compact for one layer."""
    L.require_device(K, V, W)
    kd = kv_desc(K, V, layout)
    wd = attn_desc(W)
    if wd.B != kd.B or wd.S != kd.S:
        raise ValueError(f"attention weights {tuple(W.shape)} do not match key states {tuple(K.shape)}")
    ws = workspace.get(kd.B, kd.S)
    out = bufs.out_struct()
    out.o_stride_h = kd.D  # output rows are [H, D] row-major whatever the input layout
    st = L.stream_ptr(K.device) if stream is None else stream
    if early is not None:
        seq, pub = early.next_seq(), ctypes.c_int32(0)
        rc = L.lib().rtkv_compress_layer_early(ctypes.byref(kd), ctypes.byref(wd), ctypes.byref(params),
                                               ctypes.byref(out), ws.data_ptr(), ws.numel(), st, early.ptr, seq,
                                               ctypes.byref(pub))
        L.check(rc, "rtkv_compress_layer_early")
        return LayerResult(bufs, kd.B, early if pub.value else None, seq, stream=st)
    rc = L.lib().rtkv_compress_layer(ctypes.byref(kd), ctypes.byref(wd), ctypes.byref(params), ctypes.byref(out),
                                     ws.data_ptr(), ws.numel(), st)
    L.check(rc, "rtkv_compress_layer")
    return LayerResult(bufs, kd.B, stream=st)


class PendingLayer(LayerResult):
    """A layer whose K1 and K2 are enqueued (rtkv_compress_layer_begin): stats() gives S' and the packed
    byte count (early publication, or a stream sync); finish() enqueues K4 into exactly-sized buffers."""

    def __init__(self, bufs: LayerBuffers, kd: L.KVDesc, params: L.LayerParams, workspace: "Workspace", stream: int,
                 early: Optional[EarlyStatsBuffer], seq: int, out: L.LayerOut):
        # the completion event is recorded after K4 (finish()); until then final_stats() syncs the stream
        super().__init__(bufs, kd.B, early, seq, stream=stream, record=False)
        self._kd, self._params, self._wso, self._stream, self._out = kd, params, workspace, stream, out
        self._ws = workspace.buf
        # finish()'s call, bound now: only out_rows is added after the publication
        self._finish_args = (ctypes.byref(kd), ctypes.byref(params), ctypes.byref(out))
        self._finish_tail = (self._ws.data_ptr(), self._ws.numel(), stream, early.ptr if early is not None else None,
                             seq)
        self.k_out = self.v_out = self.packed_k = self.packed_v = None
        workspace.pending = self
        self.finished = False
        self._raw = None    # the early publication as the device wrote it (converted lazily by stats())
        self._sizes = None

    def sizes(self):
        """(S'_max, packed bytes per code plane, error flags) for the output allocation: straight from the
        early publication (no conversion on this path: the device runs only K2's tail meanwhile), else
        from the synchronised statistics."""
        if self._sizes is None:
            if self._early is not None and self._stats is None:
                e = self._early.wait(self._seq, self.bufs.device)
                if e.complete:
                    self._raw = e
                    self._sizes = (e.max_kept, e.total_packed_bytes, e.error_flags)
                    return self._sizes
            st = self.stats()
            self._sizes = (st.max_kept, st.total_packed_bytes, st.error_flags)
        return self._sizes

    def stats(self) -> LayerStats:
        if self._stats is None and self._raw is not None:
            self._stats = self._checked(_early_to_stats(self._raw))
        return super().stats()

    def final_flags(self) -> Optional[int]:
        """The layer's complete RTKV_FLAG_* word as K4 published it (no stream sync), or None when it is
        not (yet) available: no early buffer, K4 not started, or overwritten by a later layer's K4."""
        return self._early.final_flags(self._seq) if self._early is not None and self.finished else None

    def wait_final_flags(self) -> int:
        """Wait (host spin, no stream sync) until this layer's K4 has started and published the layer's
        final flags, and return them; a layer without an early buffer syncs its stream instead."""
        if self._early is None or not self.finished:
            return self.final_stats_unchecked().error_flags
        flags = self._early.wait_final(self._seq, self.bufs.device)
        if flags is None:  # timed out and not in the mirror after the sync: the layer's own statistics block
            flags = self.final_stats_unchecked().error_flags
        return flags

    def _patch_out(self, kp, vp, pkp, pvp, n):
        out = self._out
        if self.bufs.emit_dequant:
            out.k_out_dev, out.v_out_dev = kp, vp
        if self.bufs.emit_packed:
            out.packed_k_dev, out.packed_v_dev, out.packed_capacity = pkp, pvp, n

    def finish(self) -> "PendingLayer":
        """Allocate K'/V' [B, S', F] and the packed codes at their exact sizes and enqueue K4 into them.
        Between the early statistics and this launch the device only runs K2's tail, so this path is
        kept short: one allocation for K'+V', one for both code planes, the begin call's LayerOut patched."""
        Sp, pb, flags = self.sizes()
        check_flags(flags)
        b = self.bufs
        dev = b.device
        kp = vp = pkp = pvp = 0
        n = 0
        if b.emit_dequant:
            kv = torch.empty((2, self.B, Sp, b.F), dtype=b.dtype, device=dev)
            kp = kv.data_ptr()
            vp = kp + self.B * Sp * b.F * kv.element_size()
            self._kv = kv
        if b.emit_packed:
            n = (max(pb, 1) + 255) // 256 * 256
            codes = torch.empty((2, n), dtype=torch.uint8, device=dev)
            pkp = codes.data_ptr()
            pvp = pkp + n
            self._codes = codes
        self._out_rows = rows = max(Sp, 1)
        self._patch_out(kp, vp, pkp, pvp, n)
        try:
            L.check(L.lib().rtkv_compress_layer_finish(*self._finish_args, rows, *self._finish_tail),
                    "rtkv_compress_layer_finish")
        finally:
            self._wso.pending = None
        self.finished = True
        if b.emit_dequant:  # views made after the launch: nothing but the allocation precedes it
            self.k_out, self.v_out = self._kv[0], self._kv[1]
            del self._kv
        if b.emit_packed:
            self.packed_k, self.packed_v = self._codes[0], self._codes[1]
            del self._codes
        self._record(self._stream)
        return self

    def final_stats_unchecked(self) -> LayerStats:
        if not self.finished and self._final is None:  # no completion event yet: K1+K2 on the layer's stream
            torch.cuda.ExternalStream(self._stream, device=self.bufs.device).synchronize()
        return super().final_stats_unchecked()

    def kv(self):
        return self.k_out, self.v_out


def compress_layer_begin(K, V, W, params: L.LayerParams, bufs: LayerBuffers, workspace: Workspace,
                         early: Optional[EarlyStatsBuffer], layout: str = "bsf", Q=None, lse=None, causal: bool = True,
                         stream: Optional[int] = None, key_bias: Optional[torch.Tensor] = None,
                         start_event: Optional[int] = None) -> PendingLayer:
    """K1 + K2 of one layer (W, or Q + lse for the fused importance mode when W is None) into the
    per-token buffers of `bufs` (LayerBuffers(..., outputs=False)); PendingLayer.finish() runs K4.
    start_event: a hipEvent_t handle (torch.cuda.Event.cuda_event) recorded right before K1."""
    L.require_device(K, V, *((Q, lse) if W is None else (W,)))
    kd = kv_desc(K, V, layout)
    if W is None:
        xd = qk_desc(Q, K, lse, causal=causal, k_layout=layout, key_bias=key_bias)
        ws = workspace.get(kd.B, kd.S, H=xd.H)
        fn, name = L.lib().rtkv_compress_layer_qk_begin, "rtkv_compress_layer_qk_begin"
    else:
        xd = attn_desc(W)
        ws = workspace.get(kd.B, kd.S)
        fn, name = L.lib().rtkv_compress_layer_begin, "rtkv_compress_layer_begin"
    if xd.B != kd.B or xd.S != kd.S:
        raise ValueError("attention input and key states disagree on B or S")
    out = bufs.out_struct()
    out.o_stride_h = kd.D
    st = L.stream_ptr(K.device) if stream is None else stream
    seq, pub = (early.next_seq(), ctypes.c_int32(0)) if early is not None else (0, ctypes.c_int32(0))
    L.check(fn(ctypes.byref(kd), ctypes.byref(xd), ctypes.byref(params), ctypes.byref(out), ws.data_ptr(), ws.numel(),
               st, early.ptr if early is not None else None, seq, ctypes.byref(pub), start_event), name)
    return PendingLayer(bufs, kd, params, workspace, st, early if pub.value else None, seq, out)

