"""Local training loop (reference ``train_model``, client1.py:96-115).

Same signature and epoch log line (``Client 1 Epoch [e/E], Average Loss: x``),
but the hot loop is device-resident: batches come from ``DeviceLoader`` (no
H2D), the per-step loss is accumulated on the device (the reference calls
``loss.item()`` twice per step, client1.py:111-112 -- one host sync each), the
head + CE loss are fused (``forward_loss``), and on GPU the whole step is a
replayed HIP graph.  One host sync per epoch.
"""
from __future__ import annotations

import time
from typing import Callable, Dict, List, Optional

import torch

from .graph import GraphedTrainStep


class fused_adam_scope:
    """Within a training step (forward + backward, then ``optimizer.step()``), let the
    model's weight-gradient GEMMs apply the optimizer's Adam step in their epilogues
    (engine/optim.py, fused mode).  Outside the scope -- gradient accumulation, a bare
    ``backward()``, data-parallel steps whose gradients must be all-reduced first --
    gradients are materialised as usual."""

    def __init__(self, model, optimizer):
        self.model = model
        self.opt = optimizer if getattr(optimizer, "can_fuse", lambda: False)() else None
        # the optimizer whose device step counter the model's training forward may advance
        # together with its dropout seed (ArenaAdam._begin(seed)); GPU arenas only
        self.step_opt = optimizer if (hasattr(optimizer, "_begin") and hasattr(model, "step_opt")
                                      and getattr(getattr(optimizer, "arena", None), "device",
                                                  torch.device("cpu")).type == "cuda") else None

    def __enter__(self):
        if self.opt is not None:
            self.model.fused_opt = self.opt
        if self.step_opt is not None:
            self.model.step_opt = self.step_opt
        return self

    def __exit__(self, *exc):
        if self.opt is not None:
            self.model.fused_opt = None
        if self.step_opt is not None:
            self.model.step_opt = None
        return False


def _one(device) -> torch.Tensor:
    """Persistent scalar 1.0 seeding ``backward`` (autograd would launch a fill per step); the
    forward is told so (``forward_loss(unit_backward=True)``: ops/kernels.py unit_grad)."""
    from ..ops.kernels import unit_grad
    return unit_grad(device)


def make_step_fn(model, optimizer, criterion=None):
    fused = criterion is None or isinstance(criterion, torch.nn.CrossEntropyLoss)

    def step(ids, mask, labels, tokens=None):
        optimizer.zero_grad()
        with fused_adam_scope(model, optimizer):
            if fused:
                loss, _ = model.forward_loss(ids, mask, labels, tokens=tokens, unit_backward=True)
            else:
                loss = criterion(model(ids, mask, tokens=tokens), labels)
            loss.backward(_one(loss.device) if loss.dtype == torch.float32 and loss.dim() == 0 else None)
        optimizer.step()
        return loss.detach()

    step.prepare = getattr(model, "prepare_replay", None)
    return step


def make_kd_step_fn(student, teacher, optimizer, temperature: float = 2.0, alpha: float = 0.5):
    """Distillation step: frozen teacher forward (no grad, eval) -> student forward with the
    distillation loss alpha * CE + (1 - alpha) * T^2 * KL(teacher || student) fused into the
    head kernel (HIP path; eager ``kd_loss`` on the torch path) -> backward -> Adam."""

    def step(ids, mask, labels, tokens=None):
        optimizer.zero_grad()
        with torch.no_grad():
            t_logits = teacher(ids, mask, tokens=tokens)
        with fused_adam_scope(student, optimizer):
            loss, _ = student.forward_loss(ids, mask, labels, tokens=tokens, kd=(t_logits, temperature, alpha),
                                           unit_backward=True)
            loss.backward(_one(loss.device) if loss.dtype == torch.float32 and loss.dim() == 0 else None)
        optimizer.step()
        return loss.detach()

    preps = [f for f in (getattr(student, "prepare_replay", None), getattr(teacher, "prepare_replay", None)) if f]
    step.prepare = (lambda: [f() for f in preps]) if preps else None
    return step


def _check_native(model):
    """Fatal-error flags of the HIP kernels (the fused LayerNorm rendezvous timeout), read at the
    epoch's one host sync."""
    if getattr(model, "impl", None) == "hip" and getattr(model, "fuse_ln", False):
        from ..ops import kernels as K
        K.check_ln_error(model.device, model.config.dim)


def train_model(model, train_loader, criterion=None, optimizer=None, num_epochs: int = 3, device=None,
                log=None, use_graph: bool = True, max_steps: Optional[int] = None,
                on_epoch: Optional[Callable] = None, teacher=None, kd_temperature: float = 2.0,
                kd_alpha: float = 0.5, grad_sync=None) -> Dict:
    """grad_sync: a ``parallel.dp.GradSync`` when this client spans k GPUs (the loader
    must then be the replica's ``DPShardLoader``); the step sums the replicas' gradients
    before Adam and the epoch loss is the client-batch mean over all replicas."""
    from .optim import ArenaAdam
    optimizer = optimizer or ArenaAdam(model)
    if log:
        log.phase("Starting model training" + (" (distillation from teacher)" if teacher is not None else ""))
    model.train()
    if teacher is not None:
        teacher.eval()
        if grad_sync is not None:
            from ..parallel.dp import make_dp_step_fn
            fn = make_dp_step_fn(model, optimizer, grad_sync, teacher, kd_temperature, kd_alpha)
        else:
            fn = make_kd_step_fn(model, teacher, optimizer, kd_temperature, kd_alpha)
    elif grad_sync is not None:
        from ..parallel.dp import make_dp_step_fn
        fn = make_dp_step_fn(model, optimizer, grad_sync)
    else:
        fn = make_step_fn(model, optimizer, criterion)
    step = GraphedTrainStep(fn, enabled=use_graph and model.device.type == "cuda",
                            bucket=getattr(model, "packed_rows", None))
    epoch_losses: List[float] = []
    steps = 0
    t0 = time.perf_counter()
    dev = model.device
    for epoch in range(num_epochs):
        loss_sum = torch.zeros((), dtype=torch.float32, device=dev)
        nb = 0
        te = time.perf_counter()
        for batch in train_loader:
            if grad_sync is not None:
                grad_sync.set_loss_scale(batch.get("loss_scale", 1.0))
            loss = step(batch["input_ids"], batch["attention_mask"], batch["labels"], batch.get("n_tokens"))
            loss_sum += loss
            nb += 1
            steps += 1
            if max_steps is not None and steps >= max_steps:
                break
        if grad_sync is not None and getattr(grad_sync, "ncomm", None) is not None:
            # the epoch's replays issued their exchanges without a host wait: a bounded native wait
            # here (RCCL async error or timeout -> ncclCommAbort + PeerFailure) instead of blocking
            # forever in the loss all-reduce / .item() below when a replica died
            grad_sync.ncomm.wait("data-parallel epoch")
        if grad_sync is not None:  # replica shares of each client-batch mean -> the mean
            import torch.distributed as dist
            dist.all_reduce(loss_sum, group=grad_sync.group)
        avg = loss_sum.item() / max(nb, 1)  # the one sync per epoch
        _check_native(model)
        dt = time.perf_counter() - te
        epoch_losses.append(avg)
        if log:
            log.info(f"Epoch [{epoch + 1}/{num_epochs}], Average Loss: {avg:.4f}",
                     batches=nb, seconds=dt, batches_per_sec=nb / dt if dt > 0 else 0.0)
        if on_epoch:
            on_epoch(epoch, avg)
        if max_steps is not None and steps >= max_steps:
            break
    if dev.type == "cuda":
        torch.cuda.synchronize()
    total = time.perf_counter() - t0
    if log:
        log.phase("Finished model training")
    return {"epoch_losses": epoch_losses, "steps": steps, "seconds": total,
            "batches_per_sec": steps / total if total > 0 else 0.0,
            "graph": step.graph is not None, "graph_error": step.failed}
