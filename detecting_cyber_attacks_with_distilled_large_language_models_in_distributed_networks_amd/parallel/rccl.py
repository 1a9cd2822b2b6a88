"""Framework-owned RCCL communicator (csrc/comm/rccl_comm.cpp).

The FedAvg data path of the reference is a TCP star with pickle + gzip
(client1.py:276-336, server.py:29-114).  ``NativeComm`` is the MI355X
replacement as a first-class object of this framework: an ``ncclComm_t``
created from a unique id that rank 0 publishes through the torch.distributed
rendezvous (TCPStore), with in-place all-reduce / broadcast / all-gather issued
on the current HIP stream (so they order with the framework's kernels and can
be captured in a HIP graph).  It binds the librccl that torch already loaded,
so one process never holds two RCCL instances.

torch.distributed (backend "nccl" = RCCL) remains the default collective path;
select this one with ``--comm rccl`` / ``FEDDDOS_COMM=rccl``.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

_OPS = {"sum": 0, "avg": 1, "max": 2}


def _torch_rccl_path() -> str:
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else "librccl.so"


class NativeComm:
    def __init__(self, rank: Optional[int] = None, world_size: Optional[int] = None):
        from ..ops._ext import ext
        self._ext = ext()
        on = dist.is_available() and dist.is_initialized()
        self.rank = rank if rank is not None else (dist.get_rank() if on else 0)
        self.world_size = world_size if world_size is not None else (dist.get_world_size() if on else 1)
        self._ext.comm_load(_torch_rccl_path())
        uid = self._ext.comm_unique_id() if self.rank == 0 else None
        if self.world_size > 1:
            if not on:
                raise RuntimeError("NativeComm with world_size > 1 needs an initialised torch.distributed "
                                   "group for the unique-id rendezvous")
            box = [bytes(uid.numpy()) if uid is not None else None]
            dist.broadcast_object_list(box, src=0)
            uid = torch.frombuffer(bytearray(box[0]), dtype=torch.uint8).clone()
        self.handle = self._ext.comm_init(self.world_size, self.rank, uid)

    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        self._ext.comm_allreduce(self.handle, t, _OPS[op])
        return t

    def broadcast_(self, t: torch.Tensor, root: int = 0) -> torch.Tensor:
        self._ext.comm_broadcast(self.handle, t, root)
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        out = torch.empty((self.world_size,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        self._ext.comm_allgather(self.handle, t.contiguous(), out)
        return out

    def close(self):
        if self.handle:
            self._ext.comm_destroy(self.handle)
            self.handle = 0
