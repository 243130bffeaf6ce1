"""Native gradient exchange: libvcg_hip's RCCL C ABI (vcg_comm_*, comm.hip) for the data-parallel step.

Replaces the NCCL communicator that reference train_video_segment_ddp.py builds through init_process_group
(:64-86) and DDP(model) (:148). One communicator per process, one process per GPU; the 128-byte RCCL id goes
from rank 0 to the other ranks through the torch.distributed store (any backend, gloo included: the store is
plumbing, the collectives are RCCL over xGMI). Collectives are asynchronous on the HIP stream they are given.
"""
import ctypes

import torch
import torch.distributed as dist

from . import _lib
from .ops import P, dt_code

UID_BYTES = 128


def unique_id():
    buf = ctypes.create_string_buffer(UID_BYTES)
    _lib.call("vcg_comm_unique_id", ctypes.addressof(buf), UID_BYTES)
    return buf.raw


class NativeComm:
    """RCCL communicator of this rank. `uid`: the id of rank 0 (default: exchanged through torch.distributed)."""

    def __init__(self, rank=None, world=None, uid=None, group=None):
        if rank is None or world is None:
            if not dist.is_initialized():
                raise RuntimeError("NativeComm: pass rank/world/uid or initialise torch.distributed first")
            rank, world = dist.get_rank(group), dist.get_world_size(group)
        if uid is None:
            obj = [unique_id() if rank == 0 else None]
            if world > 1:
                dist.broadcast_object_list(obj, src=0, group=group)
            uid = obj[0]
        buf = ctypes.create_string_buffer(bytes(uid), UID_BYTES)
        _lib.call("vcg_comm_init", int(rank), int(world), ctypes.addressof(buf), UID_BYTES)
        self.rank, self.world = rank, world

    @staticmethod
    def _sid(stream):
        return (stream or torch.cuda.current_stream()).cuda_stream

    def all_reduce(self, t, stream=None):
        """In-place SUM over the ranks of a contiguous fp32 / bf16 GPU tensor, enqueued on `stream`."""
        if not t.is_contiguous():
            raise ValueError("all_reduce needs a contiguous tensor")
        _lib.call("vcg_allreduce_bucket", P(t), t.numel(), dt_code(t.dtype), self._sid(stream))

    def broadcast(self, t, root=0, stream=None):
        if not t.is_contiguous():
            raise ValueError("broadcast needs a contiguous tensor")
        _lib.call("vcg_broadcast_bucket", P(t), t.numel(), dt_code(t.dtype), int(root), self._sid(stream))

    def close(self):
        _lib.call("vcg_comm_finalize")
