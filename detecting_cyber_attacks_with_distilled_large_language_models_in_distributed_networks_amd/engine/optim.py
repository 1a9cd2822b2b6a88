"""Single-launch Adam / AdamW over the model's flat parameter arena.

Semantics = ``torch.optim.Adam(model.parameters(), lr=2e-5)`` of the reference
(client1.py:380: betas (0.9, 0.999), eps 1e-8, weight_decay 0, bias-corrected),
with an optional decoupled weight decay (AdamW; BASELINE.json says "AdamW
step" -- identical to Adam at wd = 0).

On GPU the whole update is one HIP kernel (csrc/kernels/head_optim.hip) that
also refreshes the bf16 compute shadow; the step counter lives on the device so
the update can be replayed inside a HIP graph.  On CPU the same math runs as
flat torch ops.
"""
from __future__ import annotations

import math
from typing import Optional

import torch


class ArenaAdam:
    def __init__(self, model, lr: float = 2e-5, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, decoupled: bool = False):
        self.model = model
        self.arena = model.arena
        self.lr, self.betas, self.eps = lr, tuple(betas), eps
        self.weight_decay, self.decoupled = weight_decay, decoupled
        if weight_decay != 0.0 and getattr(model, "sparse_word_grad", False):
            model.sparse_word_grad = False  # AdamW decays every row: keep the dense word gradient
            model._hip_cache = None
        self._alloc()

    def _alloc(self):
        dev = self.arena.device
        self.m = torch.zeros_like(self.arena.master)
        self.v = torch.zeros_like(self.arena.master)
        self.step_t = torch.zeros(1, dtype=torch.int32, device=dev)
        self.host_step = 0

    def reset_state(self):
        """FedAvg rounds restart the moments (the reference re-creates Adam each run)."""
        self.m.zero_()
        self.v.zero_()
        self.step_t.zero_()
        self.host_step = 0
        if getattr(self.model, "emb_ever", None) is not None:
            self.model.emb_ever.zero_()

    def zero_grad(self, set_to_none: bool = False):
        self.model.zero_grad()

    @torch.no_grad()
    def step(self):
        A = self.arena
        if A.master.device != self.m.device:
            self._alloc()
        b1, b2 = self.betas
        self.host_step += 1
        if A.master.is_cuda:
            from ..ops import kernels as K
            K.step_inc(self.step_t, None)
            sparse = (getattr(self.model, "sparse_word_grad", False) and self.weight_decay == 0.0
                      and getattr(self.model, "emb_ever", None) is not None)
            if sparse:
                off, rows, rl = self.model.word_embedding_span()
                K.adam(A.master, A.grad, self.m, self.v, A.shadow, self.step_t, self.lr, b1, b2, self.eps,
                       self.weight_decay, self.decoupled, self.model.emb_ever, self.model.emb_now, off, rows, rl)
            else:
                if getattr(self.model, "emb_now", None) is not None and self.model.sparse_word_grad:
                    raise RuntimeError("sparse word-embedding grads need weight_decay == 0 "
                                       "(set model.sparse_word_grad = False for AdamW)")
                K.adam(A.master, A.grad, self.m, self.v, A.shadow, self.step_t, self.lr, b1, b2, self.eps,
                       self.weight_decay, self.decoupled)
            self.model.mark_shadow_synced()
            return
        t = self.host_step
        self.step_t += 1
        p, g = A.master, A.grad
        if self.weight_decay:
            if self.decoupled:
                p.mul_(1 - self.lr * self.weight_decay)
            else:
                g = g + self.weight_decay * p
        self.m.mul_(b1).add_(g, alpha=1 - b1)
        self.v.mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1 = 1 - b1 ** t
        bc2 = 1 - b2 ** t
        denom = (self.v.sqrt() / math.sqrt(bc2)).add_(self.eps)
        p.addcdiv_(self.m, denom, value=-self.lr / bc1)
        self.model.mark_shadow_synced()

    def state_dict(self):
        return {"m": self.m.cpu(), "v": self.v.cpu(), "step": int(self.step_t.item()),
                "lr": self.lr, "betas": self.betas, "eps": self.eps, "weight_decay": self.weight_decay,
                "decoupled": self.decoupled}

    def load_state_dict(self, sd):
        if getattr(self.model, "emb_ever", None) is not None:
            self.model.emb_ever.fill_(1)  # unknown history: treat every row as having state
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        self.step_t.fill_(int(sd["step"]))
        self.host_step = int(sd["step"])
