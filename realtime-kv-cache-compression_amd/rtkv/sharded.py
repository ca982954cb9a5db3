"""Sequence-sharded prefill compression: one process per GPU, ranks own contiguous token chunks.

The reference compresses one layer on one device (unified_compressor.py:95-172, called per layer
from modified_llama.py:113-117).  Here an S_total-token prefill is split into N chunks of S_local
tokens (rank j owns tokens [j*S_local, (j+1)*S_local)), and each layer runs as

  1. K1 on the rank's own W rows                       rtkv_attention_aggregation_shard
  2. all-gather of the per-token prompt mass A          4 B/token, RCCL (torch.distributed)
  3. scores / classes / selection on the whole A        rtkv_finalize_select (replicated: every rank
                                                        computes the identical global selection)
  4. per-rank output row / byte bounds                  rtkv_shard_ranges
  5. K4 on the rank's own kept K/V rows                 rtkv_quantize_rows_shard: packed codes at
                                                        their single-GPU byte offsets, dequantized
                                                        rows into a local [B, S_local, F] buffer

The selection is global (the reference's min-max normalisation and budget are over the whole
sequence, token_importance.py:71-83, selective_propagation.py:96), so step 2 is the only exchange
inside a layer.  The compressed KV of a layer is exchanged by one grouped point-to-point launch in
which each rank sends its byte ranges of the packed K/V codes and its scale/zero-point rows to every
peer (xGMI links are point-to-point, so every rank streams to all 7 peers at once instead of
hopping round a ring).  With ``overlap`` (the default) that launch is issued ``lag`` layers later,
on a communicator of its own (so it never queues in front of a later layer's all-gather of A), as
soon as the layer's rank bounds have reached the host through a non-blocking copy: the exchange of
layer l streams while layers l+1.. compute.  ``exchange()`` issues what is left and waits for all of
it.  Every rank then holds every layer's packed KV byte-identical to the single-GPU
``rtkv_compress_layer`` output.

The device stages are injected (``stages``): ``HipShardStages`` calls librtkv.so; the CPU test
suite swaps in oracle-backed stages to exercise this orchestration under gloo.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist

from . import _lib as L
from .engine import LayerBuffers, Workspace, attn_desc, kv_desc, params_from_config, prompt_length, qk_desc
from .selective_propagation import SelectiveTokenPropagator


class HipShardStages:
    """The per-rank device stages (librtkv.so), all stream-ordered and sync-free."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.ws = Workspace(self.device)
        self._qk_scratch = None

    def _stream(self):
        return L.stream_ptr(self.device)

    def aggregate(self, W, P: int, row0: int, S_total: int, A_out: torch.Tensor, params=None,
                  bufs: Optional["ShardBuffers"] = None):
        """K1 on this rank's W rows.  With the layer's params and buffers it also clears the selection scratch
        and statistics that finalize_ranges(..., zeroed=True) then uses without its memsets
        (rtkv_attention_aggregation_shard_ws)."""
        L.require_device(W, A_out)
        wd = attn_desc(W)
        if params is None:
            L.check(L.lib().rtkv_attention_aggregation_shard(ctypes.byref(wd), P, row0, S_total, A_out.data_ptr(),
                                                              self._stream()), "rtkv_attention_aggregation_shard")
            return
        ws = self.ws.get(bufs.B, bufs.S_total)
        out = bufs.out_struct()
        L.check(L.lib().rtkv_attention_aggregation_shard_ws(ctypes.byref(wd), P, row0, S_total, A_out.data_ptr(),
                                                             ctypes.byref(params), ctypes.byref(out), ws.data_ptr(),
                                                             ws.numel(), self._stream()),
                "rtkv_attention_aggregation_shard_ws")

    def finalize(self, A, a_dtype: int, params, bufs: "ShardBuffers"):
        ws = self.ws.get(bufs.B, bufs.S_total)
        out = bufs.out_struct()
        L.check(L.lib().rtkv_finalize_select(A.data_ptr(), a_dtype, bufs.B, bufs.S_total, ctypes.byref(params),
                                              ctypes.byref(out), bufs.F, L.TORCH_DTYPE_CODE[bufs.dtype],
                                              ws.data_ptr(), ws.numel(), self._stream()), "rtkv_finalize_select")

    def finalize_ranges(self, A, a_dtype: int, params, bufs: "ShardBuffers", world: int, zeroed: bool = False):
        """finalize + ranges in one call (rtkv_finalize_select_shard): the one-launch selection writes the rank
        table itself; zeroed: the layer's aggregate(..., params, bufs) cleared the scratch."""
        ws = self.ws.get(bufs.B, bufs.S_total)
        out = bufs.out_struct()
        L.check(L.lib().rtkv_finalize_select_shard(A.data_ptr(), a_dtype, bufs.B, bufs.S_total, ctypes.byref(params),
                                                    ctypes.byref(out), bufs.F, L.TORCH_DTYPE_CODE[bufs.dtype],
                                                    bufs.S_local, world, bufs.ranges.data_ptr(), int(bool(zeroed)),
                                                    ws.data_ptr(), ws.numel(), self._stream()),
                "rtkv_finalize_select_shard")

    def ranges(self, bufs: "ShardBuffers", world: int):
        L.check(L.lib().rtkv_shard_ranges(bufs.g.kept_index.data_ptr(), L.ptr(bufs.g.row_offset),
                                          bufs.g.stats.data_ptr(), bufs.B, bufs.S_total, bufs.S_local, world,
                                          bufs.ranges.data_ptr(), self._stream()), "rtkv_shard_ranges")

    def aggregate_qk(self, Q, K_prompt, lse, P: int, row0: int, causal: bool, A_out: torch.Tensor):
        """Fused importance mode on this rank's rows: A from its queries, the (broadcast) prompt keys
        [B, P, Hkv*D] and its rows' lse; row0 places the causal mask (rtkv_importance_qk_lse)."""
        L.require_device(Q, K_prompt, lse, A_out)
        qd = qk_desc(Q, K_prompt, lse, causal=causal, k_layout="bsf", row0=row0)
        n = int(L.lib().rtkv_qk_scratch_size(qd.B, qd.H, qd.S))
        if self._qk_scratch is None or self._qk_scratch.numel() < n:
            self._qk_scratch = torch.empty(n, dtype=torch.uint8, device=self.device)
        L.check(L.lib().rtkv_importance_qk_lse_ws(ctypes.byref(qd), int(P), A_out.data_ptr(), self._qk_scratch.data_ptr(),
                                                  self._qk_scratch.numel(), self._stream()), "rtkv_importance_qk_lse_ws")

    def quantize(self, K, V, layout: str, row0: int, rank: int, world: int, params, bufs: "ShardBuffers"):
        L.require_device(K, V)
        kd = kv_desc(K, V, layout)
        out = bufs.out_struct()
        out.o_stride_h = kd.D
        L.check(L.lib().rtkv_quantize_rows_shard(ctypes.byref(kd), row0, bufs.S_total, rank, world,
                                                 bufs.ranges.data_ptr(), bufs.g.labels.data_ptr(),
                                                 bufs.g.kept_index.data_ptr(), ctypes.byref(params),
                                                 ctypes.byref(out), self._stream()), "rtkv_quantize_rows_shard")


class ShardBuffers:
    """One layer on one rank: the global selection outputs (single-GPU layout, capacity S_total rows),
    the local dequantized rows, and the rank bounds table."""

    def __init__(self, B: int, S_local: int, world: int, F: int, dtype: torch.dtype, device, bits,
                 emit_dequant=True, emit_packed=True):
        self.B, self.S_local, self.world, self.F, self.dtype = B, S_local, world, F, dtype
        self.S_total = S_local * world
        dev = torch.device(device)
        self.g = LayerBuffers(B, self.S_total, F, dtype, dev, bits, emit_dequant=False, emit_packed=emit_packed)
        self.k_local = torch.empty(B, S_local, F, dtype=dtype, device=dev) if emit_dequant else None
        self.v_local = torch.empty(B, S_local, F, dtype=dtype, device=dev) if emit_dequant else None
        self.ranges = torch.zeros(B, world + 1, 2, dtype=torch.int64, device=dev)
        # host copy of the bounds for the overlapped exchange (pinned, reused every step)
        self.ranges_host = torch.zeros(B, world + 1, 2, dtype=torch.int64, pin_memory=dev.type == "cuda")

    def out_struct(self) -> L.LayerOut:
        o = self.g.out_struct()
        o.k_out_dev, o.v_out_dev = L.ptr(self.k_local), L.ptr(self.v_local)
        o.o_stride_b, o.o_stride_s, o.o_stride_h = self.S_local * self.F, self.F, self.F
        return o


@dataclass
class ShardLayer:
    """Host view of one exchanged layer: ranges[b, j] = (first row, first byte) of rank j."""
    layer_idx: int
    bufs: ShardBuffers
    ranges: torch.Tensor  # host int64 [B, world+1, 2]

    def local_rows(self, rank: int, b: int = 0) -> int:
        return int(self.ranges[b, rank + 1, 0] - self.ranges[b, rank, 0])

    def local_kv(self, rank: int):
        """This rank's dequantized kept rows, ascending token order, [B, max_b rows_b, F]."""
        n = max(self.local_rows(rank, b) for b in range(self.bufs.B))
        return self.bufs.k_local[:, :n], self.bufs.v_local[:, :n]

    def kept(self, b: int = 0) -> int:
        return int(self.ranges[b, -1, 0])


class ShardedPrefillCompressor:
    """Per-rank driver of a sequence-sharded prefill (same parameters as RealTimePrefillCompressor).

    ``enqueue_layer`` is sync-free; ``exchange`` is the one host sync + the one collective of the
    compressed KV.  ``compress_layer_kv_cache`` keeps the reference's per-layer method name for the
    rank's own token chunk (it returns the rank's dequantized rows)."""

    def __init__(self, config, group=None, stages=None, emit_packed: bool = True, emit_dequant: bool = True,
                 device=None, overlap: bool = True, lag: int = 2, collectives: str = "torch"):
        if not dist.is_initialized():
            raise RuntimeError("ShardedPrefillCompressor needs torch.distributed to be initialised")
        self.config = config
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.stages = stages if stages is not None else HipShardStages(self.device)
        self.emit_packed, self.emit_dequant = emit_packed, emit_dequant
        self.propagator = SelectiveTokenPropagator(config)
        self.bits = (int(config.low_precision_bits), int(config.medium_precision_bits),
                     int(config.high_precision_bits))
        self._bufs = {}
        self._pending: List[int] = []
        self._A = {}
        # overlapped exchange: its own communicator (own stream), layers queued with their bounds copy
        self.overlap = bool(overlap) and self.emit_packed
        self.lag = max(0, int(lag))
        self.xgroup = self.group
        if self.overlap:
            ranks = dist.get_process_group_ranks(self.group) if self.group is not None else list(range(self.world))
            self.xgroup = dist.new_group(ranks=ranks)
        # collectives: "torch" (torch.distributed on the group), "rtkv" (the C ABI's RCCL communicators:
        # rtkv_allgather_rows for A, rtkv_allgather_packed for the exchange on its own stream, the path a
        # host binding of include/rtkv.h takes) or "host" (the same exchanges staged through host memory,
        # for a group whose backend does not take device tensors, e.g. gloo: ranks sharing one GPU, or a
        # node without RCCL)
        if collectives not in ("torch", "rtkv", "host"):
            raise ValueError("collectives: 'torch', 'rtkv' or 'host'")
        self.collectives = collectives
        self._host = collectives == "host" and self.device.type == "cuda"
        self.comm = self.xcomm = self._xstream = None
        if collectives == "rtkv":
            if self.device.type != "cuda":
                raise RuntimeError("collectives='rtkv' runs RCCL: it needs ROCm devices")
            from .comm import RcclComm
            self.comm = RcclComm.from_group(self.group)
            self.xcomm = RcclComm.from_group(self.group) if self.emit_packed else None
            self._xstream = torch.cuda.Stream(self.device)
        self._prompt_keys = {}
        self._queued = []   # (layer_idx, host ranges, event) not yet exchanged
        self._issued = []   # ShardLayer whose exchange is in flight
        self._works = []

    def _peer_rank(self, j: int) -> int:
        return dist.get_global_rank(self.group, j) if self.group is not None else j

    def buffers(self, layer_idx: int, B: int, S_local: int, F: int, dtype) -> ShardBuffers:
        bf = self._bufs.get(layer_idx)
        if bf is None or (bf.B, bf.S_local, bf.F, bf.dtype) != (B, S_local, F, dtype):
            bf = ShardBuffers(B, S_local, self.world, F, dtype, self.device, self.bits, self.emit_dequant,
                              self.emit_packed)
            self._bufs[layer_idx] = bf
        return bf

    def params(self, layer_idx: int, S_total: int):
        flags = (L.EMIT_DEQUANT if self.emit_dequant else 0) | (L.EMIT_PACKED if self.emit_packed else 0)
        return params_from_config(self.config, layer_idx, prompt_length(S_total),
                                  self.propagator.get_layer_propagation_ratio(layer_idx), flags)

    def enqueue_layer(self, K, V, W, layer_idx: int, layout: str = "bsf", params=None) -> ShardBuffers:
        """K, V: this rank's [B, S_local, F] (or [B, H, S_local, D] with layout='bhsd'); W: its
        [B, H, S_local, >=P] attention rows (prompt columns P of the GLOBAL prompt)."""
        if layout == "bsf":
            B, S_local, F = K.shape
        else:
            B, H, S_local, D = K.shape
            F = H * D
        S_total = S_local * self.world
        row0 = self.rank * S_local
        P = prompt_length(S_total)
        if W.shape[0] != B or W.shape[2] != S_local or W.shape[3] < P:
            raise ValueError(f"attention rows {tuple(W.shape)} do not match the shard [B={B}, S_local={S_local}, "
                             f">= P={P}]")
        p = params if params is not None else self.params(layer_idx, S_total)
        bufs = self.buffers(layer_idx, B, S_local, F, K.dtype)
        A_local = self._A_buffers(B, S_local)[0]
        # stages with the fused finalize + ranges: K1 also clears the layer's selection scratch (no memsets)
        zeroed = hasattr(self.stages, "finalize_ranges")
        if zeroed:
            self.stages.aggregate(W, P, row0, S_total, A_local, params=p, bufs=bufs)
        else:
            self.stages.aggregate(W, P, row0, S_total, A_local)
        return self._select_and_quantize(K, V, layout, layer_idx, p, bufs, L.TORCH_DTYPE_CODE[W.dtype], zeroed)

    def enqueue_layer_qk(self, K, V, Q, lse, layer_idx: int, layout: str = "bsf", params=None,
                         causal: bool = True) -> ShardBuffers:
        """The fused importance mode on a sequence shard: K, V this rank's
        [B, S_local, F] (layout 'bsf'); Q [B, H, S_local, D] and lse [B, H, S_local] of this rank's rows.
        The prompt keys are the first P rows of the GLOBAL keys, which rank 0 holds (S_local >= P):
        they are broadcast once per layer, then every rank computes A for its own rows on MFMA."""
        if layout != "bsf":
            raise ValueError("enqueue_layer_qk takes [B, S_local, F] keys and values")
        B, S_local, F = K.shape
        S_total = S_local * self.world
        row0 = self.rank * S_local
        P = prompt_length(S_total)
        if S_local < P:
            raise ValueError(f"the prompt keys (P={P}) must lie on rank 0: S_local={S_local} < P")
        if Q.shape[0] != B or Q.shape[2] != S_local or tuple(lse.shape) != (B, Q.shape[1], S_local):
            raise ValueError(f"queries {tuple(Q.shape)} / lse {tuple(lse.shape)} do not match the shard "
                             f"[B={B}, S_local={S_local}]")
        p = params if params is not None else self.params(layer_idx, S_total)
        bufs = self.buffers(layer_idx, B, S_local, F, K.dtype)
        A_local = self._A_buffers(B, S_local)[0]
        kp = self._prompt_keys.get((B, P, F, K.dtype))
        if kp is None:
            kp = self._prompt_keys[(B, P, F, K.dtype)] = torch.empty(B, P, F, dtype=K.dtype, device=self.device)
        if self.rank == 0:
            kp.copy_(K[:, :P])
        if self.world == 1:
            pass  # the prompt keys are this rank's own
        elif self._host:
            kh = kp.cpu()
            dist.broadcast(kh, src=self._peer_rank(0), group=self.group)
            kp.copy_(kh)
        else:
            dist.broadcast(kp, src=self._peer_rank(0), group=self.group)
        self.stages.aggregate_qk(Q, kp, lse, P, row0, causal, A_local)
        return self._select_and_quantize(K, V, layout, layer_idx, p, bufs, L.F32)

    def _A_buffers(self, B: int, S_local: int):
        key = (B, S_local)
        if key not in self._A:
            S_total = S_local * self.world
            self._A[key] = (torch.empty(B, S_local, dtype=torch.float32, device=self.device),
                            torch.empty(self.world, B, S_local, dtype=torch.float32, device=self.device),
                            torch.empty(B, S_total, dtype=torch.float32, device=self.device))
        return self._A[key]

    def gather_A(self, B: int, S_local: int) -> torch.Tensor:
        """Step 2: the all-gather of every rank's A [B, S_local] into token order [B, S_total]."""
        S_total = S_local * self.world
        A_local, A_parts, A = self._A_buffers(B, S_local)
        if self.world == 1:
            return A_local  # one rank: its A is the whole row, nothing to gather
        if self.comm is not None:
            self.comm.allgather_rows(A_local, A)  # straight into token order, any B
            return A
        if self._host:
            parts = torch.empty(A_parts.numel(), dtype=A_parts.dtype)
            dist.all_gather_into_tensor(parts, A_local.reshape(-1).cpu(), group=self.group)
            A_parts.view(-1).copy_(parts)
        else:
            dist.all_gather_into_tensor(A_parts.view(-1), A_local.view(-1), group=self.group)
        if B == 1:
            return A_parts.view(1, S_total)  # rank-major = token order
        A.copy_(A_parts.permute(1, 0, 2).reshape(B, S_total))
        return A

    def _select_and_quantize(self, K, V, layout: str, layer_idx: int, p, bufs: ShardBuffers, a_dtype: int,
                             zeroed: bool = False):
        """Steps 2-5 of a layer once this rank's A is computed: all-gather, global selection, bounds,
        local quantization, and the (overlapped) exchange bookkeeping."""
        B, S_local = bufs.B, bufs.S_local
        row0 = self.rank * S_local
        A_glob = self.gather_A(B, S_local)
        fr = getattr(self.stages, "finalize_ranges", None)
        if fr is not None:  # one launch: the selection writes the rank table (B = 1, S_total <= 65536)
            fr(A_glob, a_dtype, p, bufs, self.world, zeroed=zeroed)
        else:
            self.stages.finalize(A_glob, a_dtype, p, bufs)
            self.stages.ranges(bufs, self.world)
        self.stages.quantize(K, V, layout, row0, self.rank, self.world, p, bufs)
        if self.overlap and self.world > 1:
            self._queue(layer_idx, bufs)
            self._issue(keep=self.lag)
        else:  # (one rank: nothing to exchange; the host views are made at exchange())
            self._pending.append(layer_idx)
        return bufs

    # ------------------------------------------------------------------ overlapped exchange
    def _queue(self, layer_idx: int, bufs: ShardBuffers):
        host = bufs.ranges_host
        if self.device.type == "cuda":
            host.copy_(bufs.ranges, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            host.copy_(bufs.ranges)
            ev = None
        self._queued.append((layer_idx, host, ev))

    def _issue(self, keep: int):
        # every rank issues the same layers in the same order (count-based, never completion-based),
        # as grouped point-to-point launches require
        while len(self._queued) > keep:
            layer_idx, host, ev = self._queued.pop(0)
            if ev is not None:
                ev.synchronize()  # that layer's bounds are on the host (a layer or more ago)
            sl = ShardLayer(layer_idx, self._bufs[layer_idx], host.clone())  # a snapshot: the pinned buffer is reused
            if self.xcomm is not None:
                self._rtkv_exchange(sl)
            else:
                self._works.extend(self._send_recv(sl, self.xgroup))
            self._issued.append(sl)

    def _send_recv(self, sl: ShardLayer, group):
        """One grouped launch: this rank's packed K/V byte ranges and scale/zero-point rows of the layer
        to every peer, the peers' ranges from them."""
        ops = []
        me = self.rank
        g = sl.bufs.g
        cap = sl.bufs.S_total
        sz = g.scale_zp.view(-1)
        for b in range(sl.bufs.B):
            r = sl.ranges[b]
            spans = []
            for j in range(self.world):
                b0, b1 = int(r[j, 1]), int(r[j + 1, 1])
                r0, r1 = int(r[j, 0]), int(r[j + 1, 0])
                spans.append(((b0, b1), ((b * cap + r0) * 4, (b * cap + r1) * 4)))
            for j in range(self.world):
                if j == me:
                    continue
                peer = self._peer_rank(j)
                for (lo, hi), buf in ((spans[me][0], g.packed_k), (spans[me][0], g.packed_v), (spans[me][1], sz)):
                    if hi > lo:
                        ops.append(dist.P2POp(dist.isend, buf[lo:hi], peer, group))
                for (lo, hi), buf in ((spans[j][0], g.packed_k), (spans[j][0], g.packed_v), (spans[j][1], sz)):
                    if hi > lo:
                        ops.append(dist.P2POp(dist.irecv, buf[lo:hi], peer, group))
        if self._host and ops:  # stage the byte ranges through host memory
            staged, back = [], []
            for op in ops:
                h = op.tensor.cpu() if op.op is dist.isend else torch.empty(op.tensor.shape, dtype=op.tensor.dtype)
                staged.append(dist.P2POp(op.op, h, op.peer, op.group))
                if op.op is not dist.isend:
                    back.append((op.tensor, h))
            works = dist.batch_isend_irecv(staged)
            for w in works:
                w.wait()
            for dst, h in back:
                dst.copy_(h)
            return []
        return dist.batch_isend_irecv(ops) if ops else []

    def _rtkv_exchange(self, sl: ShardLayer):
        """rtkv_allgather_packed on the exchange stream, after the layer's kernels on this stream."""
        xs = self._xstream
        xs.wait_stream(torch.cuda.current_stream(self.device))
        out = sl.bufs.g.out_struct()
        self.xcomm.allgather_packed(sl.ranges.reshape(-1).contiguous(), sl.bufs.B, sl.bufs.S_total, out,
                                    stream=xs.cuda_stream)

    def exchange(self, transfer: bool = True) -> List[ShardLayer]:
        """Finish the exchange of every layer enqueued so far and return their host views.  Overlapped
        mode: issue the layers still queued, wait for everything in flight.  Otherwise: one host read
        of every pending layer's rank bounds, then one grouped P2P launch per layer, waited once.
        ``transfer=False`` (end-of-prefill mode only) returns the host views without moving the packed
        KV: each rank then holds its own byte ranges only (bench.py times the compute this way)."""
        if not transfer and self.overlap:
            raise ValueError("exchange(transfer=False) needs overlap=False (an overlapped exchange is in flight)")
        if self.overlap:
            self._issue(keep=0)
            for w in self._works:
                w.wait()
            if self._xstream is not None:
                torch.cuda.current_stream(self.device).wait_stream(self._xstream)
            out, self._issued, self._works = self._issued, [], []
            return out + self._pending_views()  # (one rank: its layers were never queued)
        out = self._pending_views()
        if not out or self.world == 1 or not self.emit_packed or not transfer:
            return out
        if self.xcomm is not None:
            for sl in out:
                self._rtkv_exchange(sl)
            torch.cuda.current_stream(self.device).wait_stream(self._xstream)
            return out
        works = []
        for sl in out:  # one grouped launch per layer: every peer pair of the layer at once
            works.extend(self._send_recv(sl, self.group))
        for w in works:
            w.wait()
        return out

    def _pending_views(self) -> List[ShardLayer]:
        """Host views of the layers enqueued without an overlapped exchange: one host read of every layer's
        rank bounds (the single sync)."""
        layers, self._pending = list(self._pending), []
        if not layers:
            return []
        host = torch.stack([self._bufs[l].ranges for l in layers]).cpu()
        return [ShardLayer(l, self._bufs[l], host[k]) for k, l in enumerate(layers)]

    # ------------------------------------------------------------------ reference-named entry point
    def compress_layer_kv_cache(self, key_states, value_states, attention_weights, input_ids, layer_idx):
        """Rank-local twin of RealTimePrefillCompressor.compress_layer_kv_cache: compresses this rank's
        token chunk against the global selection and returns its dequantized kept rows, with the
        exchanged packed KV of the layer in ``info['shard']``.  Layers enqueued with enqueue_layer must
        be exchanged first (their results would otherwise be returned here)."""
        if self._queued or self._issued or self._pending:
            raise RuntimeError("compress_layer_kv_cache: layers enqueued with enqueue_layer are still pending; "
                               "call exchange() first")
        self.enqueue_layer(key_states, value_states, attention_weights, layer_idx)
        (sl,) = self.exchange()
        k, v = sl.local_kv(self.rank)
        info = {"layer_idx": layer_idx, "shard": sl, "rank": self.rank, "world_size": self.world,
                "original_length": sl.bufs.S_total, "max_selected_length": max(sl.kept(b) for b in range(sl.bufs.B)),
                "selection_mask": sl.bufs.g.mask.bool()}
        return k, v, info
