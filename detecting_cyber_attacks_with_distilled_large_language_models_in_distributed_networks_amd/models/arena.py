"""Flat parameter arena: fp32 master + fp32 grad + bf16 compute shadow.

One contiguous buffer per role instead of 102 separate tensors means:
  * FedAvg is ONE all-reduce over 66.4 M floats (reference: 102 pickled tensors
    gzip'd over TCP, server.py:67-114);
  * Adam is ONE kernel launch over the whole model;
  * the bf16 shadow the GEMMs read is refreshed by the optimizer in the same pass.

Each tensor starts at a 64-element (256-byte) boundary so every slice is
float4/uint4 aligned.  q/k/v weights (and biases) of a layer are laid out
back-to-back so the fused [2304, 768] QKV projection is a plain view.
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch

ALIGN = 64


def _round(n: int, a: int = ALIGN) -> int:
    return (n + a - 1) // a * a


class ParamArena:
    def __init__(self, specs: Sequence[Tuple[str, Tuple[int, ...]]], device="cpu", with_shadow: Optional[bool] = None):
        self.specs: List[Tuple[str, Tuple[int, ...]]] = list(specs)
        self.offsets: Dict[str, Tuple[int, Tuple[int, ...]]] = {}
        off = 0
        for name, shape in self.specs:
            n = math.prod(shape)
            self.offsets[name] = (off, tuple(shape))
            off += _round(n)
        self.numel = _round(off)
        self.n_params = sum(math.prod(s) for _, s in self.specs)
        device = torch.device(device)
        self.master = torch.zeros(self.numel, dtype=torch.float32, device=device)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=device)
        if with_shadow is None:
            with_shadow = device.type == "cuda"
        self.shadow = torch.zeros(self.numel, dtype=torch.bfloat16, device=device) if with_shadow else None
        self._written: set = set()

    # ---------------------------------------------------------------- views
    @property
    def device(self):
        return self.master.device

    def _slice(self, buf: torch.Tensor, name: str) -> torch.Tensor:
        off, shape = self.offsets[name]
        return buf[off:off + math.prod(shape)].view(shape)

    def view(self, name: str) -> torch.Tensor:
        return self._slice(self.master, name)

    def gview(self, name: str) -> torch.Tensor:
        return self._slice(self.grad, name)

    def sview(self, name: str) -> torch.Tensor:
        if self.shadow is None:
            raise RuntimeError("arena has no bf16 shadow (CPU arena)")
        return self._slice(self.shadow, name)

    def span(self, names: Sequence[str], which: str = "master") -> torch.Tensor:
        """Fused view over consecutive, contiguous entries (e.g. q/k/v -> [2304, 768])."""
        buf = {"master": self.master, "grad": self.grad, "shadow": self.shadow}[which]
        off0, shape0 = self.offsets[names[0]]
        total = 0
        for nm in names:
            off, shape = self.offsets[nm]
            if off != off0 + total:
                raise ValueError(f"{nm} is not contiguous with {names[0]}")
            total += math.prod(shape)
        if len(shape0) == 2:
            return buf[off0:off0 + total].view(total // shape0[1], shape0[1])
        return buf[off0:off0 + total]

    # ---------------------------------------------------------------- grad bookkeeping
    def zero_grad(self, zero_buffer: bool):
        self._written.clear()
        if zero_buffer:
            self.grad.zero_()

    def written(self, name: str) -> bool:
        """Whether the grad slot already holds a value this step (``mark_written`` without marking)."""
        return name in self._written

    def mark_written(self, name: str) -> bool:
        """Return True if the grad slot already holds a value this step (accumulate)."""
        if name in self._written:
            return True
        self._written.add(name)
        return False

    # ---------------------------------------------------------------- device / shadow
    def to(self, device) -> "ParamArena":
        device = torch.device(device)
        if device == self.master.device:
            return self
        self.master = self.master.to(device)
        self.grad = self.grad.to(device)
        if device.type == "cuda":
            self.shadow = torch.empty(self.numel, dtype=torch.bfloat16, device=device)
            self.sync_shadow()
        else:
            self.shadow = None
        return self

    def sync_shadow(self):
        """shadow <- bf16(master) (after init, load_state_dict, FedAvg)."""
        if self.shadow is None:
            return
        if self.master.is_cuda:
            from ..ops import kernels as K
            K.scale_cast(self.master, self.shadow, 1.0)
        else:
            self.shadow.copy_(self.master)

    def names(self) -> Iterable[str]:
        return (n for n, _ in self.specs)
