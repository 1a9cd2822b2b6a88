"""Process-group plumbing: one process per GPU, RCCL over xGMI (gloo on CPU).

Replaces the reference's hand-rolled TCP star (client1.py:246-336,
server.py:29-114): rendezvous is torch.distributed's TCPStore (env://,
MASTER_ADDR=127.0.0.1 by default), the data path is RCCL (backend "nccl" on
ROCm) when every rank owns a GPU, gloo otherwise.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1


_INFO: Optional[DistInfo] = None


def init_distributed(backend: Optional[str] = None, timeout_s: float = 300.0, device: Optional[str] = None) -> DistInfo:
    """Initialise from torchrun env vars; single-process when WORLD_SIZE is unset/1."""
    global _INFO
    if _INFO is not None:
        return _INFO
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = (device != "cpu") and torch.cuda.is_available()
    if use_gpu:
        n = torch.cuda.device_count()
        torch.cuda.set_device(local % max(n, 1))
        dev = torch.device("cuda", local % max(n, 1))
        if world > 1 and int(os.environ.get("LOCAL_WORLD_SIZE", str(world))) > n:
            # ranks share a GPU (gloo functional runs): no kernel may assume it owns every CU
            from ..ops import kernels as _K
            _K.set_shared_device(True)
    else:
        dev = torch.device("cpu")
    be = "none"
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        # RCCL needs one GPU per rank; FEDDDOS_BACKEND=gloo lets several clients share
        # a device (functional tests on a 1-GPU box).
        be = backend or os.environ.get("FEDDDOS_BACKEND") or ("nccl" if use_gpu else "gloo")
        kw = {}
        if be == "nccl":
            kw["device_id"] = dev
        restart = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
        if os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True" and restart != "0":
            # Elastic restart: the torchrun agent's store outlives the failed attempt, and
            # its rendezvous keys (peer addresses of the dead processes) would be reused.
            # Rendezvous the new group under a prefix of its own.
            store = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), is_master=False,
                                  timeout=datetime.timedelta(seconds=timeout_s))
            kw["store"] = dist.PrefixStore(f"fedddos_pg/{restart}", store)
        dist.init_process_group(be, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    _INFO = DistInfo(rank, world, local, be, dev)
    return _INFO


def info() -> DistInfo:
    return _INFO or DistInfo()


def barrier():
    if dist.is_available() and dist.is_initialized():
        if info().backend == "nccl":
            dist.barrier(device_ids=[info().device.index])
        else:
            dist.barrier()


def shutdown():
    global _INFO
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    _INFO = None


def all_reduce_max(x: float) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return x
    t = torch.tensor([x], dtype=torch.float64, device=info().device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_min(x: float) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return x
    t = torch.tensor([x], dtype=torch.float64, device=info().device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return float(t.item())


def broadcast_float(x: float, src: int = 0) -> float:
    """Rank ``src``'s value on every rank (identity when not distributed)."""
    if not (dist.is_available() and dist.is_initialized()):
        return x
    t = torch.tensor([x], dtype=torch.float64, device=info().device)
    dist.broadcast(t, src=src)
    return float(t.item())


def all_gather_floats(vals: List[float]) -> List[List[float]]:
    """Gather a small per-rank float vector (metrics) to every rank."""
    if not (dist.is_available() and dist.is_initialized()):
        return [list(vals)]
    t = torch.tensor(vals, dtype=torch.float64, device=info().device)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]
