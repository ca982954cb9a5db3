"""RCCL communicator of the C ABI's shard collectives (include/rtkv.h: rtkv_comm_*,
rtkv_allgather_rows, rtkv_allgather_packed).

``RcclComm.from_group(group)`` makes one RCCL communicator over the ranks of a torch.distributed
group: rank 0 draws the 128-byte id (rtkv_comm_unique_id), the group broadcasts it, every rank joins
(rtkv_comm_init).  A host without torch does the same with its own broadcast of the id.  Rank j of the
communicator is rank j of the group, i.e. shard j."""
from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist

from . import _lib as L


class RcclComm:
    def __init__(self, id_bytes: bytes, nranks: int, rank: int):
        buf = (ctypes.c_uint8 * L_COMM_ID_BYTES).from_buffer_copy(id_bytes)
        h = ctypes.c_void_p()
        L.check(L.lib().rtkv_comm_init(ctypes.byref(h), buf, L_COMM_ID_BYTES, nranks, rank), "rtkv_comm_init")
        self.handle, self.nranks, self.rank = h, nranks, rank

    @staticmethod
    def unique_id() -> bytes:
        buf = (ctypes.c_uint8 * L_COMM_ID_BYTES)()
        L.check(L.lib().rtkv_comm_unique_id(buf, L_COMM_ID_BYTES), "rtkv_comm_unique_id")
        return bytes(buf)

    @classmethod
    def from_group(cls, group=None) -> "RcclComm":
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        obj = [cls.unique_id() if rank == 0 else None]
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast_object_list(obj, src=src, group=group)
        return cls(obj[0], world, rank)

    def allgather_rows(self, a_local: torch.Tensor, a: torch.Tensor, stream=None):
        """a[b, j*S_local + i] = rank j's a_local[b, i] (fp32, [B, S_local] -> [B, nranks*S_local])."""
        B, S_local = a_local.shape
        if a_local.dtype != torch.float32 or a.dtype != torch.float32 or tuple(a.shape) != (B, S_local * self.nranks):
            raise ValueError("allgather_rows: fp32 [B, S_local] -> [B, nranks * S_local]")
        st = L.stream_ptr(a.device) if stream is None else stream
        L.check(L.lib().rtkv_allgather_rows(self.handle, a_local.data_ptr(), a.data_ptr(), B, S_local, st),
                "rtkv_allgather_rows")

    def allgather_packed(self, ranges_host: torch.Tensor, B: int, row_capacity: int, out: "L.LayerOut", stream=None):
        """Every rank's packed K/V byte ranges and scale/zp rows to every other rank, in place."""
        if ranges_host.dtype != torch.int64 or ranges_host.is_cuda or not ranges_host.is_contiguous():
            raise ValueError("allgather_packed: ranges_host must be a contiguous int64 host tensor")
        st = L.stream_ptr() if stream is None else stream
        L.check(L.lib().rtkv_allgather_packed(self.handle, ranges_host.data_ptr(), B, row_capacity,
                                              ctypes.byref(out), st), "rtkv_allgather_packed")

    def close(self):
        if self.handle:
            L.check(L.lib().rtkv_comm_destroy(self.handle), "rtkv_comm_destroy")
            self.handle = None


L_COMM_ID_BYTES = 128  # RTKV_COMM_ID_BYTES
