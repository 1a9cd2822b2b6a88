"""Stateless counter-hash dropout, bit-exact mirror of csrc/kernels/common.h.

The reference uses ATen's Philox dropout at 14 sites (hidden/attention p=0.1,
classifier p=0.3; client1.py:57,63 and HF DistilBERT).  Our kernels instead
derive every keep bit from ``hash32(site_seed, element_index >> 1)`` -- one hash per
even/odd element pair, each element comparing its own 16-bit half (low: even, high:
odd) against ``threshold(p) = round(p * 2^16)`` -- so the backward regenerates masks
instead of storing them, and the torch reference path (CPU) produces the *same* masks
for parity tests.

site_seed = hash32(counter, site) where ``counter`` is a device int32 that the
train step increments (graph-replay safe) and ``site`` identifies the dropout
call site (see ``Sites``).
"""
from __future__ import annotations

import torch

M32 = 0xFFFFFFFF


def _mulmod32(x: torch.Tensor, c: int) -> torch.Tensor:
    # (x * c) mod 2^32 without int64 overflow: split x into 16-bit halves.
    lo = x & 0xFFFF
    hi = x >> 16
    return (lo * c + (((hi * c) & 0xFFFF) << 16)) & M32


def hash32_t(seed, idx: torch.Tensor) -> torch.Tensor:
    """Vectorised hash32 over int64 tensor ``idx`` (values < 2^32)."""
    if isinstance(seed, torch.Tensor):
        seed = seed.to(torch.int64) & M32
    x = (_mulmod32(idx & M32, 0x9E3779B1) + seed) & M32
    x = x ^ (x >> 16)
    x = _mulmod32(x, 0x7FEB352D)
    x = x ^ (x >> 15)
    x = _mulmod32(x, 0x846CA68B)
    x = x ^ (x >> 16)
    return x


def hash32(seed: int, idx: int) -> int:
    def mul(a, c):
        return (a * c) & M32
    x = (mul(idx & M32, 0x9E3779B1) + (seed & M32)) & M32
    x ^= x >> 16
    x = mul(x, 0x7FEB352D)
    x ^= x >> 15
    x = mul(x, 0x846CA68B)
    x ^= x >> 16
    return x


def threshold(p: float) -> int:
    """Keep iff the element's 16-bit hash half >= threshold; p=0 -> 0 (always keep)."""
    if p <= 0.0:
        return 0
    return min(int(round(p * 65536.0)), 0xFFFF)


def keep_t(seed, idx: torch.Tensor, thr: int) -> torch.Tensor:
    """Keep bits of int64 element indices ``idx`` (common.h drop_keep)."""
    h = hash32_t(seed, idx >> 1)
    half = torch.where((idx & 1) == 1, h >> 16, h & 0xFFFF)
    return half >= thr


def site_seed(counter: int, site: int) -> int:
    return hash32(int(counter) & M32, int(site))


def keep_mask(counter: int, site: int, numel: int, p: float, device=None, offset: int = 0) -> torch.Tensor:
    """Boolean keep mask for elements [offset, offset+numel) of a dropout site."""
    thr = threshold(p)
    if thr == 0:
        return torch.ones(numel, dtype=torch.bool, device=device)
    s = site_seed(counter, site)
    idx = torch.arange(offset, offset + numel, dtype=torch.int64, device=device)
    return keep_t(s, idx, thr)


class Sites:
    """Dropout call-site ids (must match between forward and backward)."""
    EMB = 1
    HEAD = 2

    @staticmethod
    def attn(layer: int) -> int:
        return 16 + 4 * layer

    @staticmethod
    def ffn(layer: int) -> int:
        return 17 + 4 * layer
