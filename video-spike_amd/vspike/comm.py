"""The C-ABI gradient exchange (vs_comm_*, include/vspike.h) for hosts that want RCCL without
torch.distributed's process group, e.g. a native trainer calling libvspike directly.

Replaces the implicit DDP all-reduce of the reference's accelerate setup (src/train.py:61-64).
The Python training path uses vspike.dp.GradExchange over torch.distributed (backend "nccl" =
RCCL); this class exposes the same in-place bucket all-reduce through the library's own RCCL
communicator, enqueued on torch's current stream.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib as L

COMM_ID_BYTES = 128


class RcclComm:
    """One RCCL communicator of this process on the current device."""

    def __init__(self, world: int, rank: int, unique_id: bytes):
        if len(unique_id) != COMM_ID_BYTES:
            raise ValueError(f"unique_id must be {COMM_ID_BYTES} bytes")
        self.world, self.rank = int(world), int(rank)
        buf = ctypes.create_string_buffer(unique_id, COMM_ID_BYTES)
        h = ctypes.c_void_p()
        L.check(L.lib().vs_comm_init(ctypes.byref(h), buf, self.world, self.rank), "vs_comm_init")
        self.handle = h.value

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(COMM_ID_BYTES)
        L.check(L.lib().vs_comm_unique_id(buf), "vs_comm_unique_id")
        return buf.raw

    @classmethod
    def from_process_group(cls, group=None) -> "RcclComm":
        """Rank 0 of a torch.distributed group makes the id; every rank builds its communicator."""
        import torch.distributed as dist
        obj = [cls.unique_id() if dist.get_rank(group) == 0 else None]
        dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        return cls(dist.get_world_size(group), dist.get_rank(group), obj[0])

    def allreduce_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over ranks of a contiguous f32 / bf16 device tensor, on the current stream."""
        L.require_device(t)
        if not t.is_contiguous():
            raise ValueError("allreduce_ needs a contiguous tensor")
        L.check(L.lib().vs_comm_allreduce_bucket(self.handle, t.data_ptr(), t.numel(), L.dtype_code(t.dtype),
                                                 L.stream()), "vs_comm_allreduce_bucket")
        return t

    def close(self):
        if getattr(self, "handle", None):
            L.lib().vs_comm_finalize(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
