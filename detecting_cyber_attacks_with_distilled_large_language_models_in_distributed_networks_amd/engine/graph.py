"""HIP-graph capture of the whole training step (forward + backward + Adam).

At B32/S128 one step is ~150 kernel launches; replaying them as one hipGraph
removes the per-launch host cost and all Python/autograd overhead from the
steady state (the MI355X replacement for a tracing compiler).  The dropout
seed counter and the Adam step count live on the device and are advanced by
kernels inside the graph, so every replay is a fresh, correct step.

Protocol: the first ``warmup`` calls run eagerly (they are real training steps
on the real batches, and they populate allocator pools / workspaces); the next
call captures, then replays the capture for its own batch.  Batches whose shape
differs from the captured one (the last partial batch, drop_last=False) run
eagerly.
"""
from __future__ import annotations

from typing import Callable, Dict, Optional

import torch


class GraphedTrainStep:
    def __init__(self, step_fn: Callable[[torch.Tensor, torch.Tensor, torch.Tensor], torch.Tensor],
                 warmup: int = 2, enabled: bool = True):
        self.step_fn = step_fn
        self.warmup = warmup
        self.enabled = enabled and torch.cuda.is_available()
        self.calls = 0
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.shape = None
        self.static: Dict[str, torch.Tensor] = {}
        self.static_loss: Optional[torch.Tensor] = None
        self.failed: Optional[str] = None

    def __call__(self, ids: torch.Tensor, mask: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        self.calls += 1
        if not self.enabled or self.failed:
            return self.step_fn(ids, mask, labels)
        if self.graph is not None:
            if ids.shape != self.shape:
                return self.step_fn(ids, mask, labels)
            self.static["ids"].copy_(ids)
            self.static["mask"].copy_(mask)
            self.static["labels"].copy_(labels)
            self.graph.replay()
            return self.static_loss
        if self.calls <= self.warmup:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                loss = self.step_fn(ids, mask, labels)
            torch.cuda.current_stream().wait_stream(s)
            return loss
        # capture
        self.shape = ids.shape
        self.static = {"ids": ids.clone(), "mask": mask.clone(), "labels": labels.clone()}
        g = torch.cuda.CUDAGraph()
        try:
            torch.cuda.synchronize()
            with torch.cuda.graph(g):
                self.static_loss = self.step_fn(self.static["ids"], self.static["mask"], self.static["labels"])
        except Exception as e:  # pragma: no cover - capture support varies by op
            self.failed = f"{type(e).__name__}: {e}"
            torch.cuda.synchronize()
            return self.step_fn(ids, mask, labels)
        self.graph = g
        g.replay()
        return self.static_loss
