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

Failure semantics (the reference's 300 s socket timeouts, client1.py:22 / server.py:10): an
eager collective is followed by a bounded native wait (csrc/comm/rccl_comm.cpp fd_comm_wait)
that polls the stream together with ``ncclCommGetAsyncError``.  An RCCL-reported error or a
timeout aborts the communicator (``ncclCommAbort``, which also releases the stuck collective)
and raises ``PeerFailure`` instead of hanging the rank forever.  Collectives issued during HIP
graph capture are not waited on (the graph's replay is; see ``wait``).
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

from .health import PeerFailure

_OPS = {"sum": 0, "avg": 1, "max": 2}
COMM_TIMEOUT = 1001  # csrc/comm/rccl_comm.cpp FD_COMM_TIMEOUT


def _torch_rccl_path() -> str:
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else "librccl.so"


class CommAborted(PeerFailure):
    """A collective of ``NativeComm`` failed or timed out; the communicator was aborted."""

    def __init__(self, code: int, msg: str, where: str):
        RuntimeError.__init__(self, f"RCCL {where}: {msg} (code {code}); communicator aborted")
        self.dead = []  # RCCL does not name the lost peer
        self.code = code


class NativeComm:
    """group: a torch.distributed sub-group (e.g. one data-parallel client's replicas): the
    communicator then spans that group only, ranked by group rank; its unique id travels over the
    group from the group's first rank.  Every rank of the WORLD must construct the communicators of
    the groups it belongs to in the same order (as with ``dist.new_group``)."""

    def __init__(self, rank: Optional[int] = None, world_size: Optional[int] = None,
                 timeout_s: Optional[float] = None, group=None):
        from ..ops._ext import ext
        self._ext = ext()
        # bounded wait per eager collective (FEDDDOS_COMM_TIMEOUT_S; reference socket timeout 300 s)
        self.timeout_s = float(timeout_s if timeout_s is not None else os.environ.get("FEDDDOS_COMM_TIMEOUT_S", 300.0))
        on = dist.is_available() and dist.is_initialized()
        src = 0
        if group is not None:
            if not on:
                raise RuntimeError("NativeComm(group=...) needs an initialised torch.distributed")
            self.rank, self.world_size = dist.get_rank(group), dist.get_world_size(group)
            src = dist.get_global_rank(group, 0)
        else:
            self.rank = rank if rank is not None else (dist.get_rank() if on else 0)
            self.world_size = world_size if world_size is not None else (dist.get_world_size() if on else 1)
        self._ext.comm_load(_torch_rccl_path())
        uid = self._ext.comm_unique_id() if self.rank == 0 else None
        if self.world_size > 1:
            if not on:
                raise RuntimeError("NativeComm with world_size > 1 needs an initialised torch.distributed "
                                   "group for the unique-id rendezvous")
            box = [bytes(uid.numpy()) if uid is not None else None]
            dist.broadcast_object_list(box, src=src, group=group)
            uid = torch.frombuffer(bytearray(box[0]), dtype=torch.uint8).clone()
        self.handle = self._ext.comm_init(self.world_size, self.rank, uid)

    def _live(self):
        if not self.handle:
            raise RuntimeError("NativeComm was aborted or closed")
        return self.handle

    def wait(self, where: str = "collective"):
        """Bounded wait for the work issued so far on the current stream (skipped while the
        stream is being captured into a graph).  RCCL async error or timeout -> abort + raise."""
        if torch.cuda.is_current_stream_capturing():
            return
        code, msg = self._ext.comm_wait(self._live(), int(self.timeout_s * 1000))
        if code:
            self.abort()
            raise CommAborted(int(code), msg, where)

    def check(self):
        """Raise (after aborting) if RCCL recorded an asynchronous error on this communicator."""
        code, msg = self._ext.comm_async_error(self._live())
        if code:
            self.abort()
            raise CommAborted(int(code), msg, "async error")

    def all_reduce_(self, t: torch.Tensor, op: str = "sum", wait: bool = True) -> torch.Tensor:
        self._ext.comm_allreduce(self._live(), t, _OPS[op])
        if wait:
            self.wait("all_reduce")
        return t

    def broadcast_(self, t: torch.Tensor, root: int = 0, wait: bool = True) -> torch.Tensor:
        self._ext.comm_broadcast(self._live(), t, root)
        if wait:
            self.wait("broadcast")
        return t

    def all_gather(self, t: torch.Tensor, wait: bool = True) -> torch.Tensor:
        out = torch.empty((self.world_size,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        self._ext.comm_allgather(self._live(), t.contiguous(), out)
        if wait:
            self.wait("all_gather")
        return out

    def abort(self):
        """ncclCommAbort: release the communicator without waiting for (dead) peers."""
        if self.handle:
            h, self.handle = self.handle, 0
            self._ext.comm_abort(h)

    def close(self):
        if self.handle:
            self._ext.comm_destroy(self.handle)
            self.handle = 0
