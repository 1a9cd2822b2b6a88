"""Federated averaging.

Reference (server.py:67-79): gather exactly NUM_CLIENTS pickled state_dicts,
``base[key] += m_i[key]; base[key] /= N`` (unweighted, in place on client 0's
dict), then broadcast the mean back (server.py:81-114) -- ~20 s of gzip + TCP
per round for 265 MB.

Here: every client's fp32 master weights already sit in one flat arena, so a
round is ONE collective (``all_reduce(SUM)`` over 66.4 M floats on RCCL/xGMI)
followed by one fused HIP pass that applies the 1/N (or 1/sum-of-weights)
scale and re-casts the bf16 compute shadow.  Options the reference lacks:
sample-count weighting (pre-scale by n_k) and partial participation (a
non-participating / dropped client contributes weight 0 and receives the
average of the live clients).

``aggregate_state_dicts`` keeps the reference's server-side API for
state_dict lists (floating tensors only -- an int64 buffer would make the
reference's in-place ``/=`` raise).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

from .comm import info


def _dist_on() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


@torch.no_grad()
def broadcast_model(model, src: int = 0, comm=None):
    """Make every client start from rank ``src``'s weights (identical init).

    comm: optional ``parallel.rccl.NativeComm`` (framework-owned RCCL communicator)."""
    if _dist_on():
        if comm is not None:
            comm.broadcast_(model.arena.master, root=src)
        else:
            dist.broadcast(model.arena.master, src=src)
    model.sync_shadow(force=True)


@torch.no_grad()
def fedavg_(model, weight: float = 1.0, participate: bool = True, comm=None) -> float:
    """In-place FedAvg of ``model`` across all ranks; returns the total weight.

    weight:      this client's aggregation weight (1 = unweighted, n_k = sample-weighted)
    participate: False -> this client's update is dropped this round (fault injection /
                 partial participation); it still receives the aggregate.
    comm:        optional ``parallel.rccl.NativeComm``; default is the torch.distributed group.
    """
    A = model.arena
    w = float(weight) if participate else 0.0
    if not _dist_on():
        if w == 0.0:
            return 0.0
        model.sync_shadow(force=True)
        return w
    dev = A.master.device
    wt = torch.tensor([w], dtype=torch.float64, device=dev)
    use_native = comm is not None and A.master.is_cuda

    def allreduce(t):
        if use_native:
            comm.all_reduce_(t, "sum")
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)

    allreduce(wt)
    total = float(wt.item())
    if total <= 0:
        raise RuntimeError("FedAvg round with no participating clients")
    if A.master.is_cuda:
        from ..ops import kernels as K
        if w != 1.0:
            K.scale_cast(A.master, None, w)          # pre-scale (0 drops the update)
        allreduce(A.master)
        K.scale_cast(A.master, A.shadow, 1.0 / total)  # fused 1/W scale + bf16 shadow refresh
        model.mark_shadow_synced()
    else:
        if w != 1.0:
            A.master.mul_(w)
        dist.all_reduce(A.master, op=dist.ReduceOp.SUM)
        A.master.mul_(1.0 / total)
        model.sync_shadow(force=True)
    return total


def aggregate_state_dicts(states: Sequence[Dict[str, torch.Tensor]], weights: Optional[Sequence[float]] = None,
                          num_clients: Optional[int] = None):
    """server.py:67-79 semantics: None unless exactly ``num_clients`` models; mean of float tensors."""
    if num_clients is not None and len(states) != num_clients:
        return None
    if not states:
        return None
    ws = list(weights) if weights is not None else [1.0] * len(states)
    tot = float(sum(ws))
    out = OrderedDict()
    for k, v0 in states[0].items():
        if torch.is_floating_point(v0):
            acc = torch.zeros_like(v0, dtype=torch.float32)
            for s, w in zip(states, ws):
                acc += s[k].to(acc.device, torch.float32) * w
            out[k] = (acc / tot).to(v0.dtype)
        else:
            out[k] = v0.clone()
    return out
