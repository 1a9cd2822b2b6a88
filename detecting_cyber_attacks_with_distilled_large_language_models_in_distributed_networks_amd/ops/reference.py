"""Pure-PyTorch (fp32, autograd) reference of every fused kernel.

Used (a) as the CPU execution path (gloo plumbing runs, CI without a GPU) and
(b) as the numerics oracle in the kernel tests.  Semantics match the HF
DistilBERT code the reference calls ([ext] modeling_distilbert.py)
and the kernels' dropout hash (ops/dropout.py), so for a given (counter, site)
both paths drop exactly the same elements.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from .dropout import keep_mask


# Numerics experiments only (scripts/curve_bisect.py): round every tensor the HIP path stores in
# bf16 (activations between kernels, the pre-LN sums, attention probabilities before P.V) to bf16
# here too -- in the forward and, through the casts' autograd, in the backward.
BF16_STORAGE = False


def _st(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.bfloat16).to(t.dtype) if BF16_STORAGE and t.dtype == torch.float32 else t


def dropout_ref(x: torch.Tensor, p: float, counter: Optional[int], site: int) -> torch.Tensor:
    if p <= 0.0 or counter is None:
        return x
    keep = keep_mask(counter, site, x.numel(), p, device=x.device).view(x.shape)
    return torch.where(keep, x / (1.0 - p), torch.zeros_like(x))


def linear_ref(x, w, b=None):
    return _st(F.linear(x, w, b))


def gelu_ref(x):
    return _st(F.gelu(x))  # exact erf form (HF GELUActivation)


def add_ln_ref(x, r, gamma, beta, eps=1e-12, p=0.0, counter=None, site=0):
    """LN(dropout(x) + r) over the last dim."""
    z = dropout_ref(x, p, counter, site)
    if r is not None:
        z = z + r
    return _st(F.layer_norm(_st(z), (z.shape[-1],), gamma, beta, eps))


def embedding_ref(ids, word, pos, gamma, beta, eps=1e-12, p=0.0, counter=None, site=0):
    """Dropout(LN(word[ids] + pos[s])) -> [B*S, D]."""
    B, S = ids.shape
    z = word[ids.reshape(-1)] + pos[:S].repeat(B, 1)
    y = F.layer_norm(z, (z.shape[-1],), gamma, beta, eps)
    return _st(dropout_ref(y, p, counter, site))


def attention_ref(qkv: torch.Tensor, mask: torch.Tensor, B: int, S: int, H: int, p: float = 0.0,
                  counter=None, site: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """qkv [B*S, 3*H*64] -> (ctx [B*S, H*64], lse [B, H, S])."""
    D = H * 64
    q, k, v = qkv.view(B, S, 3, H, 64).permute(2, 0, 3, 1, 4)  # each [B, H, S, 64]
    scores = (q / math.sqrt(64)) @ k.transpose(-1, -2)
    keymask = (mask.view(B, 1, 1, S) == 0)
    scores = scores.masked_fill(keymask, float("-inf"))
    lse = torch.logsumexp(scores, dim=-1)
    probs = torch.softmax(scores, dim=-1)
    probs = _st(dropout_ref(probs, p, counter, site))
    ctx = _st((probs @ v).permute(0, 2, 1, 3).reshape(B * S, D))
    return ctx, lse


def head_ref(hidden: torch.Tensor, B: int, S: int, W, b, p=0.3, counter=None, site=0):
    """hidden [B*S, D] -> logits [B, 2] via CLS -> Dropout -> Linear."""
    D = hidden.shape[-1]
    cls = hidden.view(B, S, D)[:, 0, :]
    cls = dropout_ref(cls, p, counter, site)
    return F.linear(cls, W, b)


def layer_ref(x, P: dict, B, S, H, mask, eps=1e-12, p_attn=0.0, p_hidden=0.0, counter=None,
              attn_site=0, ffn_site=0):
    """One DistilBERT TransformerBlock (post-LN), x [B*S, D]."""
    qkv = linear_ref(x, P["qkv_w"], P["qkv_b"])
    ctx, _ = attention_ref(qkv, mask, B, S, H, p_attn, counter, attn_site)
    ao = linear_ref(ctx, P["o_w"], P["o_b"])
    h = add_ln_ref(ao, x, P["ln1_w"], P["ln1_b"], eps)
    u = linear_ref(h, P["l1_w"], P["l1_b"])
    f = linear_ref(gelu_ref(u), P["l2_w"], P["l2_b"])
    return add_ln_ref(f, h, P["ln2_w"], P["ln2_b"], eps, p_hidden, counter, ffn_site)
