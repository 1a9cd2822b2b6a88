"""Thin, allocation-aware Python wrappers over the gfx950 kernel extension.

All functions expect GPU tensors; shapes are validated in the C++ binding
before any launch.  Scratch buffers (split-K slabs, column-sum partials) come
from a per-device workspace cache that only grows, so steady-state steps do no
allocation and the whole step can be captured into a HIP graph.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ._ext import ext
from .dropout import threshold

D_MODEL = 768
LN_GRID = 256  # must match csrc/kernels/norm.hip (partial-sum blocks of the embedding backward)
LN_BWD_PARTS = 512  # upper bound on the LN backward's partial-sum blocks (csrc/kernels/norm.hip)

_WS = {}
# Outgrown workspaces are kept alive, never freed: a HIP graph captured earlier (another
# packed-row bucket, another batch shape) still holds their addresses, and returning them to
# the caching allocator would let a later allocation alias memory that graph writes on replay.
_WS_RETIRED = []


def workspace(device, name: str, numel: int, dtype=torch.float32) -> torch.Tensor:
    key = (str(device), name, dtype)
    t = _WS.get(key)
    if t is None or t.numel() < numel:
        if t is not None:
            _WS_RETIRED.append(t)
            numel_alloc = max(numel, t.numel() + t.numel() // 2)  # grow geometrically: few retirements
        else:
            numel_alloc = numel
        t = torch.empty(max(numel_alloc, 1), dtype=dtype, device=device)
        _WS[key] = t
    return t[:numel]


def _drop(p: float):
    thr = threshold(p)
    return thr, (1.0 / (1.0 - p) if thr else 1.0)


# ------------------------------------------------------------------ GEMMs
EPI_BF16, EPI_BIAS, EPI_BIAS_GELU, EPI_GELU_BWD, EPI_ADD = 0, 1, 2, 3, 4
EPI_LN, EPI_LN_BWD = 6, 7

# Small-M GEMMs (the pruned last block's [CLS] rows, M = 64): split over K into fp32 slabs and
# reduced by one epilogue launch (csrc/kernels/splitk.hip) -- the single-pass kernels would run
# the whole K loop on the dozen CUs its 64 x 64 tiles cover.  FD_SPLITK_SMALLM=0: off.
import os as _os
SPLITK_MAX_M = 64 if _os.environ.get("FD_SPLITK_SMALLM", "1") != "0" else 0
# FD_SPLITK_MINK: split only problems with K >= this (the shorter ones run single-pass)
SPLITK_MIN_K = int(_os.environ.get("FD_SPLITK_MINK", "0"))


def _splitk_ok(M: int, N: int, K: int) -> bool:
    return 0 < M <= SPLITK_MAX_M and N % 64 == 0 and K % 64 == 0 and K >= SPLITK_MIN_K


def _splitk(epi, x, wt, y, **kw):
    """One split-K GEMM + epilogue (``ext().gemm_splitk``) on the shared slab workspace (slabs
    are consumed by the epilogue launch right behind the GEMM on the same stream).  b_mn=True:
    ``wt`` is the weight W [K, N] itself (y = epi(x W))."""
    M, N = x.shape[0], (wt.shape[1] if kw.get("b_mn") else wt.shape[0])
    ws = workspace(x.device, "splitk_small", 256 * M * N // max(1, ((M + 63) // 64) * (N // 64)) + M * N)
    return ext().gemm_splitk(epi, x, wt, y, ws, **kw)


# The LayerNorm-fused GEMMs touch the NEXT launch's weight while they wait for their row statistics
# (csrc/kernels/gemm.hip pf_issue; cold weights cost the QKV forward ~4 us, profiles/r4_cold_operands.txt).
# FD_LN_PREFETCH=0: off (A/B).
LN_PREFETCH = _os.environ.get("FD_LN_PREFETCH", "1") != "0"


def _pf(t):
    return t if (LN_PREFETCH and t is not None and t.is_cuda and t.is_contiguous()) else None


# FD_NOGRAD_SKIP_U=0: forwards without autograd write the FFN pre-activation u anyway (A/B knob)
NOGRAD_SKIP_U = _os.environ.get("FD_NOGRAD_SKIP_U", "1") != "0"


def linear_fwd(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], gelu: bool = False, prefetch=None,
               keep_u: bool = True):
    """y = x w^T + b (bf16), optionally also returning u (pre-GELU) with y = gelu(u).  prefetch: the
    next launch's weight, touched by the epilogue (``LN_PREFETCH``).  keep_u=False (a forward without
    autograd): u is not written (returned as None) -- 2 bytes per FFN element less."""
    M, N = x.shape[0], w.shape[0]
    y = torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
    if _splitk_ok(M, N, x.shape[1]):
        if gelu:
            u = torch.empty_like(y)
            _splitk(EPI_BIAS_GELU, x, w, y, bias=b, aux=u)
            return y, u
        _splitk(EPI_BIAS if b is not None else EPI_BF16, x, w, y, bias=b)
        return y
    if gelu:
        u = torch.empty_like(y) if keep_u or not NOGRAD_SKIP_U else None
        ext().gemm(0, EPI_BIAS_GELU, x, w, y, b, u, None, None, False, None, _pf(prefetch))
        return y, u
    ext().gemm(0, EPI_BIAS if b is not None else EPI_BF16, x, w, y, b, None, None, None, False, None, _pf(prefetch))
    return y


def linear_dx(dy: torch.Tensor, w: torch.Tensor, gelu_u: Optional[torch.Tensor] = None,
              res: Optional[torch.Tensor] = None,
              colsum: Optional[tuple] = None, aux_out: Optional[torch.Tensor] = None, prefetch=None) -> torch.Tensor:
    """dx = dy w  [* gelu'(u)]  [+ res]  (bf16).

    The product reads the weight ``w`` [N_out, N_in] itself as an MN-major B operand ("NN",
    transposing LDS fragment reads): no W^T copy is kept (a per-step W^T refresh lost its A/B,
    profiles/r4_ab_dx_layouts.txt).
    colsum = (deferred colsum jobs, out, accumulate): the GEMM epilogue also leaves the column
    sums of dx per M tile (the producer-bias gradient) as a deferred job, instead of a separate
    column-sum pass over dx.  aux_out (with gelu_u): the epilogue also writes gelu(gelu_u) there
    -- the forward's activation, bitwise.  Returns dx."""
    M, N = dy.shape[0], w.shape[1]
    dx = torch.empty(M, N, dtype=torch.bfloat16, device=dy.device)
    B, bmn, kind = w, True, 1
    epi = EPI_GELU_BWD if gelu_u is not None else (EPI_ADD if res is not None else EPI_BF16)
    ao = aux_out if gelu_u is not None else None
    if colsum is not None and epi == EPI_BF16:
        raise ValueError("fused column sums need a GELU' / residual epilogue")
    if _splitk_ok(M, N, dy.shape[1]):
        if colsum is not None:
            jobs, out, acc = colsum
            cs = workspace(dy.device, f"colsum_job{len(jobs)}", ((M + 31) // 32) * N)
            _, nblk = _splitk(epi, dy, B, dx, aux=gelu_u, aux_out=ao, res=res, colsum=cs, b_mn=bmn)
            jobs.append((cs, [out], nblk, N, N, acc))
            return dx
        _splitk(epi, dy, B, dx, aux=gelu_u, aux_out=ao, res=res, b_mn=bmn)
        return dx
    if colsum is not None:
        jobs, out, acc = colsum
        ws = workspace(dy.device, f"colsum_job{len(jobs)}", ((M + 127) // 128) * N)
        nblk = ext().gemm_colsum(epi, dy, B, dx, gelu_u, res, ws, ao, kind, _pf(prefetch))
        if nblk:
            jobs.append((ws, [out], nblk, N, N, acc))
            return dx
        # this shape's tile has no fused column sums: plain GEMM, then the separate pass
        ext().gemm(kind, epi, dy, B, dx, None, gelu_u, res, None, False, ao, _pf(prefetch))
        _colsum_pass(dx, out, acc, jobs)
        return dx
    ext().gemm(kind, epi, dy, B, dx, None, gelu_u, res, None, False, ao, _pf(prefetch))
    return dx


def linear_dw(dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor, accumulate: bool = False,
              adam=None) -> torch.Tensor:
    """out[N_out, N_in] (fp32) (+)= dy^T x (split-K fp32 slabs + a deterministic reduce launch).
    adam = (state, hyper) from ``ArenaAdam.fused_args``: apply Adam to the finished gradient
    instead of storing it."""
    M, N = dy.shape[1], x.shape[1]
    ws = workspace(dy.device, "splitk", 8 * M * N)
    st, hp = adam if adam is not None else ([], [])
    ext().gemm_dw(dy, x, out, ws, accumulate, st, hp)
    return out


def linear_dw2(dy0: torch.Tensor, x0: torch.Tensor, out0: torch.Tensor, dy1: torch.Tensor, x1: torch.Tensor,
               out1: torch.Tensor, accumulate: bool = False, adam=None, jobs: Optional[list] = None):
    """Two weight gradients that become ready together, one launch: out_i (+)= dy_i^T x_i
    (adam: fused optimizer step for both, see ``linear_dw``).  jobs: a deferred-reduce list --
    a split-K launch leaves its fp32 slabs in a buffer of its own and ``dw_flush`` reduces
    every deferred gradient of the backward in one launch (same z order: bitwise equal)."""
    n = out0.numel() + out1.numel()
    defer = False
    if jobs is not None and adam is None:
        planned = ext().gemm_dw2_splits(dy0.shape[1], x0.shape[1], dy1.shape[1], x1.shape[1], dy0.shape[0])
        defer = planned > 1
    # a deferred launch keeps its slabs until the flush: a buffer of its own, sized to the plan
    ws = workspace(dy0.device, f"splitk_def{len(jobs)}", planned * n) if defer else \
        workspace(dy0.device, "splitk", 8 * n)
    st, hp = adam if adam is not None else ([], [])
    splits = ext().gemm_dw2(dy0, x0, out0, dy1, x1, out1, ws, accumulate, st, hp, defer)
    if splits:
        s0 = splits * out0.numel()
        jobs.append((ws[:s0], out0, splits, accumulate))
        jobs.append((ws[s0:s0 + splits * out1.numel()], out1, splits, accumulate))


DW_BATCH_MAX = 32  # problems per all-layer weight-gradient launch (csrc/kernels/gemm.hip DWB_MAXP)


# The rest of the optimizer step (biases, LayerNorms, embeddings, head, the flagged word rows) run
# by extra blocks of the all-layer dW launch, on the CUs its last round of tiles leaves idle,
# instead of two launches after it; the qkv bias by the tiles that sum its gradient
# (engine/optim.py ArenaAdam.rest_args; FD_ADAM_IN_DW=0: step() launches it).
ADAM_IN_DW = _os.environ.get("FD_ADAM_IN_DW", "1") != "0"


# Problem order of the all-layer dW launch (A/B): 0 = backward order as recorded (the pruned last
# block's problems first), 1 = reversed (forward block order).
DWB_ORDER = int(_os.environ.get("FD_DWB_ORDER", "0"))


def linear_dw_batch(jobs: list, adam=None, cfg: int = -1, opt=None):
    """Every weight gradient of a backward in one launch per 32 problems: for each job
    (dy [K, M], x [K, N], out [M, N] fp32, accumulate[, bias]) out (+)= dy^T x, and the
    optional fp32 [M] bias (+)= the column sums of dy (``DW_QKV_BIAS``).  No split-K: each
    output tile runs the whole token dimension (deterministic, no slabs, no reduce).
    adam: a callable grads -> (state, hyper) (``ArenaAdam.fused_args``): apply the optimizer
    step to each finished gradient tile instead of storing it.  opt (with adam): the optimizer
    (``ArenaAdam``) -- the last launch also runs the rest of its step (``ADAM_IN_DW``)."""
    if DWB_ORDER == 1 and len(jobs) <= DW_BATCH_MAX:
        jobs = jobs[::-1]  # (forward block order: the pruned block's problems last)
    starts = list(range(0, len(jobs), DW_BATCH_MAX))
    for i in starts:
        chunk = jobs[i:i + DW_BATCH_MAX]
        outs = [j[2] for j in chunk]
        st, hp = adam(outs) if adam is not None else ([], [])
        bias = [j[4] if len(j) > 4 else None for j in chunk]
        rest = None
        if adam is not None and opt is not None and ADAM_IN_DW and i == starts[-1]:
            # the qkv biases summed by this launch are updated by its tiles when it also finishes
            # the step: mark them, then hand the rest of the step to the launch
            sums = [b for b in bias if b is not None]
            done0 = len(opt._done)
            opt.mark_done(sums)
            rest = opt.rest_args()
            if rest is None:
                del opt._done[done0:]  # (step() updates them after all)
        if any(b is not None for b in bias):
            none = torch.empty(0, dtype=torch.float32, device=outs[0].device)
            bias = [b if b is not None else none for b in bias]
        else:
            bias = []
        ext().gemm_dw_batch([j[0] for j in chunk], [j[1] for j in chunk], outs, [int(j[3]) for j in chunk],
                            st, hp, cfg, bias, *(rest if rest is not None else ([], [])))


# The qkv bias gradient from the all-layer dW launch itself: the qkv weight gradient's tiles of the
# first column block sum dqkv's columns while their K loops read it (gemm.hip GemmParams::acol),
# instead of a separate column-sum pass over every block's dqkv.  FD_DW_QKV_BIAS=0: the pass.
DW_QKV_BIAS = _os.environ.get("FD_DW_QKV_BIAS", "1") != "0"


def dw_flush(jobs: list):
    """Reduce every deferred split-K weight gradient in one launch."""
    if jobs:
        ext().splitk_reduce_batched([j[0] for j in jobs], [j[1] for j in jobs], [j[2] for j in jobs],
                                    [int(j[3]) for j in jobs])
        jobs.clear()


def _colsum_pass(x, out, accumulate, jobs):  # (linear_dx's `colsum` argument shadows colsum())
    return colsum(x, out, accumulate, jobs)


def colsum(x: torch.Tensor, out: torch.Tensor, accumulate: bool = False, jobs: Optional[list] = None) -> torch.Tensor:
    """out (+)= column sums of x.  With ``jobs`` (a deferred-colsum list) only the per-block
    partials are computed now, into a slot of their own; ``colsum_flush`` finalises them."""
    N = out.numel()
    T = x.numel() // N
    if jobs is None:
        ws = workspace(x.device, "colsum", ((T + 31) // 32) * N)
        ext().colsum_bf16(x, out, ws, accumulate, False)
        return out
    ws = workspace(x.device, f"colsum_job{len(jobs)}", ((T + 31) // 32) * N)
    nblk = ext().colsum_bf16(x, out, ws, accumulate, True)
    jobs.append((ws, [out], nblk, N, N, accumulate))
    return out


def gather_rows2(a: torch.Tensor, b: torch.Tensor, idx: torch.Tensor):
    """(a[idx], b[idx]) for two same-shape bf16 [T, D] matrices, one launch (idx int64, device)."""
    oa = torch.empty(idx.numel(), a.shape[1], dtype=a.dtype, device=a.device)
    ob = torch.empty_like(oa)
    ext().gather_rows2(a, b, oa, ob, idx)
    return oa, ob


def scatter_rows2(a: torch.Tensor, b: torch.Tensor, idx: torch.Tensor, nsrc: int, T: int):
    """Two zero-filled [T, D] matrices with rows idx[k] = a[k] / b[k] for k < nsrc (idx ascending
    over those k), one launch."""
    oa = torch.empty(T, a.shape[1], dtype=a.dtype, device=a.device)
    ob = torch.empty_like(oa)
    ext().scatter_rows2(a, b, oa, ob, idx, nsrc)
    return oa, ob


def colsum_partials_batched(pending: list, jobs: list):
    """Partials of several deferred bf16 column sums -- pending = [(x, out, accumulate)] -- in ONE
    launch, each appended to ``jobs`` exactly as ``colsum(x, out, accumulate, jobs)`` would
    (bitwise the same partials; ``colsum_flush`` finalises them)."""
    if not pending:
        return
    xs, parts, ns = [], [], []
    for x, out, acc in pending:
        N = out.numel()
        T = x.numel() // N
        ws = workspace(x.device, f"colsum_job{len(jobs)}", ((T + 31) // 32) * N)
        jobs.append((ws, [out], (T + 31) // 32, N, N, acc))
        xs.append(x)
        parts.append(ws)
        ns.append(N)
    ext().colsum_bf16_batched(xs, parts, ns)
    pending.clear()


def colsum_flush(jobs: list):
    """Finalise every deferred column sum in one launch (bitwise = the immediate path)."""
    if jobs:
        ext().colsum_batched([j[0] for j in jobs], [j[1] for j in jobs], [j[2] for j in jobs],
                             [j[3] for j in jobs], [j[4] for j in jobs], [int(j[5]) for j in jobs])
        jobs.clear()


# ------------------------------------------------------------------ unpadded layout
def pack(mask: torch.Tensor, ids: torch.Tensor, rows: int, step=None, seed=None, cls_rows=None, cls_rmap=None):
    """(row_map int32 [rows], cu int32 [B+1], ids_packed int64 [rows]) of a [B, S] batch: the
    real tokens in order (filler rows: row_map -1, id of position 0) -- one launch, which also
    advances the optional int32 counters ``step`` / ``seed`` (what ``step_inc`` would launch) and
    writes cu[b] as int64 into ``cls_rows[b]`` when given (the pruned last block's row list) and the
    padded row of packed row cu[b] into ``cls_rmap[b]`` (int32; its dropout-hash rows)."""
    B = mask.shape[0]
    row_map = torch.empty(rows, dtype=torch.int32, device=mask.device)
    cu = torch.empty(B + 1, dtype=torch.int32, device=mask.device)
    ids_packed = torch.empty(rows, dtype=torch.int64, device=mask.device)
    m = mask if mask.dtype != torch.bool else mask.to(torch.uint8)
    ext().pack(m.contiguous(), ids.contiguous(), row_map, cu, ids_packed, step, seed, cls_rows, cls_rmap)
    return row_map, cu, ids_packed


# ------------------------------------------------------------------ attention
def mask_bias(mask: torch.Tensor) -> torch.Tensor:
    m = mask.contiguous()
    if m.dtype == torch.bool:
        m = m.to(torch.uint8)
    bias = torch.empty(m.shape, dtype=torch.float32, device=m.device)
    ext().mask_to_bias(m, bias)
    return bias


def attn_keep_bits(B, S, H, p, device, short: bool = False) -> Optional[torch.Tensor]:
    """Buffer for the dropout keep bits the S <= 128 attention forward hands to its backward
    (which then reads them instead of re-hashing every probability twice); None when unused.
    short: a varlen batch at S > 128 whose sequences all fit the S <= 128 kernels."""
    if not threshold(p) or (S > 128 and not short):
        return None
    return torch.empty(B * H * 256, dtype=torch.int64, device=device)


# The S <= 128 attention kernel writes the pruned block's compact [CLS] rows itself (gather_rows2
# folded into the attention launch); FD_ATTN_CLS_COMPACT=0 restores the separate gather.
ATTN_CLS_COMPACT = _os.environ.get("FD_ATTN_CLS_COMPACT", "1") != "0"


def attn_cls_compact_ok(S: int, short: bool = False) -> bool:
    return ATTN_CLS_COMPACT and (S <= 128 or short) and _os.environ.get("FD_ATTN_S128", "1") != "0"


def attn_fwd(qkv, kbias, B, S, H, seed, site, p, cu=None, dmask=None, q_live: int = 0, cls=None, short=False):
    """cu (int32 [B+1]): varlen mode -- qkv/ctx hold packed sequences (rows cu[b]..cu[b+1]-1);
    the kernel zeroes ctx's filler rows past cu[B] itself.  dmask (``attn_keep_bits``): also
    record the dropout keep bits for ``attn_bwd``.

    cls = (x, Bp) (q_live 1, ``attn_cls_compact_ok(S)``): also return ctx[cls_rows] and
    x[cls_rows] as [Bp, D] -- sequence b's [CLS] row in compact row b, rows B..Bp-1 copies of
    row 0 (the pruned block's ``cls_rows`` layout) -- written by the attention blocks that own the
    rows.  Returns (ctx, lse) or (ctx, lse, cxc, xc).

    Varlen at S > 128 (csrc/kernels/attention.hip split_mode): sequences of <= 128 tokens run on the
    S <= 128 whole-row kernel, longer ones on the 64-row kernel (FD_ATTN_SPLIT=0: the latter alone);
    short=True (every sequence has <= 128 tokens, known on the host) skips the 64-row launch."""
    rows = qkv.shape[0] if cu is not None else B * S
    ctx = torch.empty(rows, H * 64, dtype=torch.bfloat16, device=qkv.device)
    lse = torch.empty(B, H, S, dtype=torch.float32, device=qkv.device)
    thr, sc = _drop(p)
    if cls is None:
        # q_live > 0 (S <= 128): only the first q_live query rows of each sequence are computed
        ext().attn_fwd(qkv, kbias, ctx, lse, B, S, H, seed, site, thr, sc, cu, dmask if thr else None, q_live,
                       split=2 if short and cu is not None else -1)
        return ctx, lse
    x, Bp = cls
    cxc = torch.empty(Bp, H * 64, dtype=torch.bfloat16, device=qkv.device)
    xc = torch.empty_like(cxc)
    ext().attn_fwd(qkv, kbias, ctx, lse, B, S, H, seed, site, thr, sc, cu, dmask if thr else None, q_live,
                   cxc, xc, x, split=2 if short and cu is not None else -1)
    return ctx, lse, cxc, xc


# QKV projection + S <= 128 attention forward in ONE launch (csrc/kernels/gemm.hip).  FD_FUSE_QKV_ATTN:
#   0: the two launches;
#   1: gemm_attn_fwd_kernel -- the QKV tiles hand off to the attention items (write-through stores +
#      tagged granules; needs the LayerNorm exchange epoch to advance per forward, RunCtx.fuse_ln):
#      step-neutral, the one-round GEMM's tiles all finish together;
#   2 (default): seq_attn_fwd_kernel -- one block per (sequence, head) projects its own Q / K / V
#      rows (live rows only) straight into the attention's LDS images: 25.3 vs 25.8 us per layer,
#      -2.4 us per step over 6 interleaved 200-step pairs (profiles/r6_ab_fused_qkv_attention.txt).
# Both bitwise the two launches (tests/test_qkv_attn_gpu.py).
FUSE_QKV_ATTN = int(_os.environ.get("FD_FUSE_QKV_ATTN", "2"))


# Short batches at S > 128 (data.PackedTokens): the producer-GEMM fusions of the S <= 128 attention take
# them only with FD_ATTN_SHORT_FUSED=1 -- at the distillation config (seq256 bs64, 18 attention layers
# per step) the per-(sequence, head) QKV projection measured +112 us per step and the out-projection
# dX in the backward +16 us against the separate GEMMs (profiles/r6_ab_attn_short_fused.txt); the keep
# bits hand-off and the compact [CLS] rows apply either way.
ATTN_SHORT_FUSED = _os.environ.get("FD_ATTN_SHORT_FUSED", "0") != "0"


def qkv_attn_ok(M: int, D: int, S: int, short: bool = False) -> bool:
    """Shapes the fused QKV + attention launch takes (csrc/binding.cpp gemm_attn_fwd); short: a varlen
    batch at S > 128 whose sequences all have <= 128 tokens (the per-(sequence, head) mode 2 only,
    ``ATTN_SHORT_FUSED``)."""
    short = short and ATTN_SHORT_FUSED
    return (FUSE_QKV_ATTN and not _SHARED_DEVICE and _os.environ.get("FD_ATTN_S128", "1") != "0"
            and (S in (64, 128) or (short and FUSE_QKV_ATTN == 2 and S % 64 == 0 and S <= 512)) and D % 64 == 0 and M > 0 and M * 3 * D * 2 < 2 ** 31
            and ((M + 127) // 128) * (3 * D // 192) <= QA_FLAGS)


def qkv_attn_fwd(x, w, b, kbias, B, S, H, seed, site, p, cu=None, dmask=None, q_live: int = 0, cls=None,
                 xsite: int = 0, prefetch=None, mode=None, short: bool = False):
    """``linear_fwd(x, w, b)`` then ``attn_fwd(qkv, ...)`` as one launch (``qkv_attn_ok``).  xsite:
    this launch's call site within the current exchange epoch (``ln_xsite``; the fused launches
    keep their own granules, so a block's LayerNorm site number can be reused); mode: 1 / 2 (see
    ``FUSE_QKV_ATTN``; None = that setting, or 1 when it is off).  Mode 2 leaves qkv's filler rows
    past cu[B] zero (nothing reads them).  Returns
    (qkv, ctx, lse) or, with cls = (x_res, Bp), (qkv, ctx, lse, cxc, xc)."""
    M, D = x.shape[0], H * 64
    qkv = torch.empty(M, 3 * D, dtype=torch.bfloat16, device=x.device)
    rows = M if cu is not None else B * S
    ctx = torch.empty(rows, D, dtype=torch.bfloat16, device=x.device)
    lse = torch.empty(B, H, S, dtype=torch.float32, device=x.device)
    thr, sc = _drop(p)
    stats, cnt, err = _ln_state(x.device, M, D)
    kw = {}
    if cls is not None:
        xr, Bp = cls
        kw = dict(cxc=torch.empty(Bp, D, dtype=torch.bfloat16, device=x.device), xres=xr)
        kw["xc"] = torch.empty_like(kw["cxc"])
    ext().gemm_attn_fwd(x, w, b, qkv, kbias, ctx, lse, B, S, H, seed, site, thr, sc, cu, dmask if thr else None,
                        q_live, stats, cnt, err, int(xsite), prefetch=_pf(prefetch),
                        mode=int(mode if mode is not None else (FUSE_QKV_ATTN or 1)),
                        split=2 if short and cu is not None else -1, **kw)
    if cls is None:
        return qkv, ctx, lse
    return qkv, ctx, lse, kw["cxc"], kw["xc"]


# The S <= 128 attention backward that computes its own dO -- the out-projection's dX for the
# (sequence, head)'s rows and columns -- inside the launch (csrc/kernels/gemm.hip
# attn_bwd_proj_kernel): one launch and one dctx round trip less per block -- 26.7 vs 19.4 + 9.1 us per
# layer, -12 us per step over 10 interleaved 200-step pairs (profiles/r6_ab_attn_bwd_proj.txt).
# FD_FUSE_ATTN_BWD=0: the out-projection dX GEMM + the attention backward.
FUSE_ATTN_BWD = int(_os.environ.get("FD_FUSE_ATTN_BWD", "1"))


# the pruned block's compact [CLS] form of it (FD_FUSE_ATTN_BWD_CLS=0: the split-K out-projection dX +
# the attention backward there)
FUSE_ATTN_BWD_CLS = int(_os.environ.get("FD_FUSE_ATTN_BWD_CLS", "1"))


def attn_bwd_proj_ok(S: int, cls: bool = False, short: bool = False) -> bool:
    short = short and ATTN_SHORT_FUSED
    return (bool(FUSE_ATTN_BWD) and (not cls or bool(FUSE_ATTN_BWD_CLS)) and (S in (64, 128) or short)
            and _os.environ.get("FD_ATTN_S128", "1") != "0")


def _dx_splits(M: int, N: int, K: int) -> int:
    """The K splits ``linear_dx`` runs an M x N x K product with: the split-K slabs of the small-M
    GEMMs (csrc/kernels/gemm.hip fd_gemm_f32_splits' pick), else 1 (one chain)."""
    if not _splitk_ok(M, N, K):
        return 1
    tiles = ((M + (63 if M <= 64 else 127)) // (64 if M <= 64 else 128)) * (N // 64)
    nkt, s = K // 64, 1
    for c in range(1, nkt + 1):
        if nkt % c == 0 and tiles * c <= 256 and nkt // c >= 2:
            s = c
    return s


def attn_bwd_proj(qkv, kbias, ctx, lse, dy, w, B, S, H, seed, site, p, cu=None, dmask=None, dresc=None,
                  short: bool = False):
    """``attn_bwd(qkv, kbias, ctx, lse, linear_dx(dy, w), ...)`` as one launch (S <= 128): dy [rows, K]
    is the out-projection's output gradient, w [K, H 64] its weight.  dresc (the pruned block's
    compact form, q_live 1): dy is the [CLS] rows' gradient [Bp, K] and, as in ``attn_bwd``, the launch
    also scatters dresc into the full layout.  Bitwise the two-launch path (including the split-K
    summation order of the small-M product).  Returns dqkv, or (dqkv, dres)."""
    dqkv = torch.empty_like(qkv)
    thr, sc = _drop(p)
    splits = _dx_splits(dy.shape[0], w.shape[1], dy.shape[1])
    if dresc is None:
        ext().attn_bwd_proj(qkv, kbias, ctx, lse, dy, w, dqkv, B, S, H, seed, site, thr, sc, cu,
                            dmask if thr else None, splits, split=2 if short and cu is not None else -1)
        return dqkv
    dres = torch.empty_like(ctx)
    ext().attn_bwd_proj(qkv, kbias, ctx, lse, dy, w, dqkv, B, S, H, seed, site, thr, sc, cu,
                        dmask if thr else None, splits, dresc.contiguous(), dres,
                        split=2 if short and cu is not None else -1)
    return dqkv, dres


def attn_bwd(qkv, kbias, ctx, lse, dctx, B, S, H, seed, site, p, cu=None, dmask=None, q_live: int = 0, dresc=None,
             short=False):
    """dmask: the keep bits recorded by the matching ``attn_fwd`` (same seed / site / p).

    dresc ([Bp, D], q_live 1, ``attn_cls_compact_ok(S)``): ``dctx`` is the compact [CLS]
    gradient [Bp, D] (row b = sequence b's [CLS] row, every other row's dO 0) and the launch also
    scatters ``dresc`` into the full layout -- returns (dqkv, dres) with dres = what
    ``scatter_rows2(dctx, dresc, cls_rows, B, rows)[1]`` gives; otherwise dqkv."""
    dqkv = torch.empty_like(qkv)  # varlen: filler rows zeroed by the dQ kernel
    delta = workspace(qkv.device, "attn_delta", B * H * S)
    thr, sc = _drop(p)
    if dresc is None:
        ext().attn_bwd(qkv, kbias, ctx, lse, dctx.contiguous(), delta, dqkv, B, S, H, seed, site, thr, sc, cu,
                       dmask if thr else None, q_live, split=2 if short and cu is not None else -1)
        return dqkv
    dres = torch.empty_like(ctx)
    ext().attn_bwd(qkv, kbias, ctx, lse, dctx.contiguous(), delta, dqkv, B, S, H, seed, site, thr, sc, cu,
                   dmask if thr else None, q_live, dresc.contiguous(), dres, split=2 if short and cu is not None else -1)
    return dqkv, dres


# ------------------------------------------------------------------ layernorm / embedding
def ln_fwd(x, r, gamma, beta, eps, seed, site, p, row_map=None):
    """row_map (int32 [T]): packed row -> padded row, for the dropout hash only."""
    T = x.numel() // gamma.numel()
    y = torch.empty_like(x)
    mean = torch.empty(T, dtype=torch.float32, device=x.device)
    rstd = torch.empty(T, dtype=torch.float32, device=x.device)
    thr, sc = _drop(p)
    ext().ln_fwd(x, r, gamma, beta, y, mean, rstd, eps, seed, site, thr, sc, row_map if thr else None)
    return y, mean, rstd


def ln_bwd(dy, x, r, gamma, mean, rstd, dgamma, dbeta, dbias, seed, site, p, accumulate=False, row_map=None,
           jobs: Optional[list] = None, zin: bool = False):
    """jobs: deferred-colsum list -> the dgamma/dbeta/dbias partials wait for ``colsum_flush``.
    zin: ``x`` is the saved pre-LN sum z of a LayerNorm-fused GEMM (``r`` must be None); dropout
    only masks the returned dx."""
    D = gamma.numel()
    T = x.numel() // D
    dz = torch.empty_like(x)
    thr, sc = _drop(p)
    dx = torch.empty_like(x) if thr else None
    key = "ln_part" if jobs is None else f"ln_part_job{len(jobs)}"
    ws = workspace(x.device, key, LN_BWD_PARTS * 3 * D)
    nblk = ext().ln_bwd(dy.contiguous(), x, r, gamma, mean, rstd, dz, dx, dgamma, dbeta, dbias, ws, seed, site, thr,
                        sc, accumulate, row_map if thr else None, jobs is not None, zin)
    if jobs is not None:
        jobs.append((ws, [dgamma, dbeta, dbias], nblk, 3 * D, D, accumulate))
    return dz, (dx if dx is not None else dz)


# ------------------------------------------------------------------ LayerNorm fused into a GEMM
LN_STATE_ROWS = 32768  # row capacity of the exchange state (grown if a call needs more)


def _ln_state(device, M: int, N: int):
    """(stats, cnt, err) of the LayerNorm-fused GEMM (csrc/kernels/gemm.hip gemm_ln_kernel):
    the tagged row-statistic granules, the exchange epoch and the timeout flag.  Zeroed once;
    the epoch is advanced by ``emb_fwd`` (the first launch of every model forward) or by
    ``ln_epoch_advance`` (graph replays reuse the same state)."""
    key = (_dev_key(device), "ln_state", N)
    st = _WS.get(key)
    rows = max(M, LN_STATE_ROWS)
    if st is None or st[3] < M:
        if st is not None:
            _WS_RETIRED.append(st)
        # the epoch survives a regrow: a granule tag must never repeat on the same state
        epoch = st[1] if st is not None else torch.zeros(2, dtype=torch.int32, device=device)
        err = st[2] if st is not None else torch.zeros(1, dtype=torch.int32, device=device)
        # (+ QA_FLAGS granules of the fused QKV + attention launch, then LN2_FLAGS at the tail: the
        # two-K-half tiles' exchange flags, csrc/binding.cpp)
        st = (torch.zeros(2 * (rows + 256) * (N // 64) + QA_FLAGS + LN2_FLAGS, dtype=torch.int64, device=device),
              epoch, err, rows)
        _WS[key] = st
    return st[:3]


LN_XSITES = 128  # csrc/kernels/adam_epi.h FD_LN_XSITES: exchange call sites per epoch
LN2_FLAGS = 512  # csrc/binding.cpp gemm_ln: flag granules of the two-K-half tiles
QA_FLAGS = 1024  # csrc/binding.cpp gemm_attn_fwd: tile granules of the fused QKV + attention launch
# Two-K-half LayerNorm-fused GEMMs (csrc/kernels/gemm.hip gemm_ln2_kernel, K >= FD_GEMM_LN2_MINK):
# the fp32 partial-tile exchange buffer (FD_LN2=0: never passed, the one-pass kernels run)
LN2 = _os.environ.get("FD_LN2", "1") != "0"


def _ln2_xbuf(device):
    # (<= 128 tile pairs of 2 x 128 x 64 fp32 partials, or of 2 x 256 x 64 for the 256-row tiles)
    return workspace(device, "ln2_xbuf", 128 * 2 * 16384) if LN2 else None


def ln_xsite(layer: int, which: int, backward: bool) -> int:
    """Exchange call site of a model's LayerNorm-fused launch: forward out_lin / lin2 of block
    ``layer`` -> 2 * layer + which; the backward ones (lin1 dX / qkv dX) 64 + 2 * layer + which.
    Unique within one forward + backward (the epoch advances once per forward).  At most 125:
    site 127 would let a granule tag wrap to the 0 of a freshly zeroed granule."""
    if not 0 <= layer < 31 or which not in (0, 1):
        raise ValueError(f"no LayerNorm exchange site for block {layer} / {which}")
    return (64 if backward else 0) + 2 * layer + which


def ln_epoch(device, N: int = D_MODEL) -> torch.Tensor:
    """The exchange epoch tensor (int32), for ``emb_fwd(ln_epoch=...)``."""
    return _ln_state(device, 1, N)[1]


def ln_stats(device, N: int = D_MODEL) -> torch.Tensor:
    """The exchange's granule buffer (int64), for ``emb_fwd(ln_stats=...)``: the epoch launch
    zeroes it whenever the 32-bit granule tags are about to repeat (every 2^25 epochs)."""
    return _ln_state(device, 1, N)[0]


def ln_epoch_advance(device, N: int = D_MODEL):
    """Start a new exchange epoch (one small launch): callers of ``linear_ln_fwd`` /
    ``linear_dx_ln_bwd`` that do not run a model forward (tests, scripts) use this."""
    ln_epoch(device, N)[:1].add_(1)


def check_ln_error(device, N: int = D_MODEL):
    """Raise if a LayerNorm-fused launch's row-block rendezvous ever timed out: its statistics
    (and every output after it) are wrong.  One host sync; call it at epoch / eval boundaries."""
    if ln_error_flag(device, N):
        raise RuntimeError("a LayerNorm-fused GEMM timed out waiting for its row block's statistics "
                           "(other work held the GPU's CUs?): the results of this run are invalid; "
                           "rerun with FD_FUSE_LN=0 if the GPU is shared")


def _xsite(device, N, xsite):
    if xsite is None:  # a standalone call: a fresh epoch of its own
        ln_epoch_advance(device, N)
        return 0
    return int(xsite)


LN_MAX_TILES = 256  # csrc/kernels/gemm.hip: the fused grid is one resident round of the CUs


_CUS = {}


def _cu_count() -> int:
    dev = torch.cuda.current_device() if torch.cuda.is_available() else -1
    if dev not in _CUS:
        _CUS[dev] = torch.cuda.get_device_properties(dev).multi_processor_count if dev >= 0 else LN_MAX_TILES
    return _CUS[dev]


# Tile configuration of the LayerNorm-fused GEMMs (csrc/kernels/gemm.hip fd_gemm_ln): -1 = the
# launcher's default (FD_GEMM_LN_CFG or its measured pick); tests pin the others.
LN_CFG = -1

# Several processes on one GPU (gloo functional runs, FEDDDOS_BACKEND=gloo): another process's
# kernels can hold the CUs a fused-LN tile's peers need, and two such grids then block each other
# until the rendezvous times out (measured: tests/test_dp_gpu.py, two replicas on one MI355X).  Set
# by parallel/comm.py init_distributed; the separate LayerNorm kernels run instead.
_SHARED_DEVICE = False


def set_shared_device(shared: bool) -> None:
    global _SHARED_DEVICE
    _SHARED_DEVICE = bool(shared)


_LN2_FLAGS = 512  # csrc/binding.cpp gemm_ln: the two-K-half exchange's flag granules


def ln_fusable(M: int, N: int, concurrent_collectives: bool = False, K=None) -> bool:
    """Whether a LayerNorm-fused GEMM of M rows x N (= hidden) columns runs as one resident
    round (its row blocks exchange statistics, so no tile may wait on an undispatched peer):
    at most one 128 x 64 tile per CU, no other process on the device, and no collective of this
    process in flight beside it (``concurrent_collectives``: a data-parallel client's gradient
    all-reduces overlapping the backward -- RCCL's kernels hold CUs and LDS while they wait on a
    slower replica, so a fused tile's row-block peers might not get a CU until the 0.25 s
    rendezvous timeout).  Otherwise the plain GEMMs + separate LayerNorm kernels.
    K (an int or the inner sizes of every GEMM the caller will fuse): the 256-row two-K-half route
    is counted only where the launcher takes it (gemm.hip fd_gemm_ln ``ln2_ok``: K % 128 == 0, no
    FD_GEMM_LN_CFG / LN_CFG override, and the exchange flags of binding.cpp's capacity) -- a shape
    judged fusable here never makes ``gemm_ln`` raise instead of falling back."""
    if _SHARED_DEVICE or concurrent_collectives:
        return False
    tiles = ((M + 127) // 128) * (N // 64)
    ks = () if K is None else ((K,) if isinstance(K, int) else tuple(K))
    ln2_ok = (LN2 and N % 128 == 0 and all(k % 128 == 0 for k in ks) and LN_CFG < 0
              and int(_os.environ.get("FD_GEMM_LN_CFG", "-1")) < 0
              and ((M + 127) // 128) * (N // 128) * 2 <= _LN2_FLAGS)
    if ln2_ok:  # (gemm.hip fd_gemm_ln: 256-row two-K-half tiles past the 128-row round)
        tiles = min(tiles, ((M + 255) // 256) * (N // 64))
    return N % 64 == 0 and N <= 2048 and tiles <= min(LN_MAX_TILES, _cu_count())


def ln_set_diag(diag: int):
    """Tests / profiling only: FD_GEMM_LN_DIAG at run time (64 forces the rendezvous timeout)."""
    ext().gemm_ln_set_diag(int(diag))


def ln_error_flag(device, N: int = 768) -> int:
    """Nonzero if a fused-LN launch's row-block rendezvous ever timed out (never expected)."""
    st = _WS.get((_dev_key(device), "ln_state", N))
    return 0 if st is None else int(st[2].item())


def _dev_key(device) -> str:
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return str(d)


def linear_ln_fwd(x, w, b, res, gamma, beta, eps, seed, site, p, row_map=None, keep_z: bool = True, xsite=None,
                  prefetch=None):
    """y = LN(dropout(x w^T + b) + res) in ONE launch (the N = hidden GEMM's epilogue does the
    bias, dropout, residual and LayerNorm).  Returns (y, z, mean, rstd): z = the bf16 pre-LN sum
    (what the backward reads; None with keep_z=False), mean / rstd fp32 per row.  xsite: the
    launch's exchange call site (``ln_xsite``) within the current epoch; None = a new epoch."""
    M, N = x.shape[0], w.shape[0]
    y = torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
    z = torch.empty_like(y) if keep_z else None
    mean = torch.empty(M, dtype=torch.float32, device=x.device)
    rstd = torch.empty(M, dtype=torch.float32, device=x.device)
    thr, sc = _drop(p)
    if _splitk_ok(M, N, x.shape[1]):
        _splitk(EPI_LN, x, w, y, bias=b, res=res, gamma=gamma, beta=beta, mean=mean, rstd=rstd, z=z, eps=eps,
                seed=seed, site=site, thr=thr, dscale=sc, row_map=row_map if thr else None)
        return y, z, mean, rstd
    stats, cnt, err = _ln_state(x.device, M, N)
    xs = _xsite(x.device, N, xsite)
    ext().gemm_ln(False, x, w, y, b, res, gamma, beta, mean, rstd, z, None, None, stats, cnt, err, eps, seed, site,
                  thr, sc, row_map if thr else None, LN_CFG, xs, False, _ln2_xbuf(x.device), _pf(prefetch))
    return y, z, mean, rstd


# The pruned training step's head inside the output-LayerNorm split-K epilogue of the last block
# (csrc/kernels/splitk.hip sk_head_row): one launch fewer than head_ln_bwd; FD_HEAD_IN_SK=0: off.
HEAD_IN_SK = _os.environ.get("FD_HEAD_IN_SK", "1") != "0"


def head_in_sk_ok(M: int, N: int, K: int) -> bool:
    return HEAD_IN_SK and FUSE_HEAD and N == 768 and _splitk_ok(M, N, K)


_HEAD_TICKETS = {}


def _head_ticket(dev) -> torch.Tensor:
    """The fused head's ticket counter (int32 [1], zeroed once and only ever advanced: a launch's
    last row block holds ticket % rows == rows - 1), one per device."""
    t = _HEAD_TICKETS.get(dev)
    if t is None:
        t = _HEAD_TICKETS[dev] = torch.zeros(1, dtype=torch.int32, device=dev)
    return t


def linear_ln_fwd_head(x, w, b, res, gamma, beta, eps, seed, site, p, row_map, hW, hb, head_site, p_head, labels,
                       B, own, kd, dW, db, acc_head, dgamma, dbeta, dbias, acc_ln, jobs, loss_acc=None):
    """``linear_ln_fwd`` on the pruned [CLS] rows (split-K) with the head fused into its epilogue:
    per row the head logits / loss / dlogits, the head gradient of the row (the loss's upstream
    gradient is 1) and the LayerNorm backward of it.  The head dW / db, the loss mean (and the
    running ``loss_acc``) and the LayerNorm affine gradients are column sums of per-row partials,
    appended to the deferred ``jobs``; the loss mean itself is finished inside the launch (its last
    row block sums the row losses in row order), so ``loss`` is valid as soon as the forward returns
    (it used to be filled only by the backward's deferred sums).
    Returns (y, z, mean, rstd, (logits, loss, dz, dx))."""
    M, N = x.shape[0], w.shape[0]
    dev = x.device
    y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    z = torch.empty_like(y)
    mean = torch.empty(M, dtype=torch.float32, device=dev)
    rstd = torch.empty(M, dtype=torch.float32, device=dev)
    thr, sc = _drop(p)
    hthr, hsc = _drop(p_head)
    logits = torch.empty(B, 2, dtype=torch.float32, device=dev)
    dlogits = torch.empty(B, 2, dtype=torch.float32, device=dev)
    loss = torch.empty((), dtype=torch.float32, device=dev)
    dz = torch.empty_like(y)
    dx = torch.empty_like(y) if thr else None
    n = len(jobs)
    colpart = workspace(dev, f"ln_colpart_job{n}", M * 3 * N)
    hpart = workspace(dev, f"head_part_job{n}", M * 2 * N)
    dbpart = workspace(dev, f"head_db_job{n}", M * 2)
    lpart = workspace(dev, f"head_loss_job{n}", M)
    t, kT, alpha = kd if kd is not None else (None, 1.0, 1.0)
    if t is not None:
        t = t.detach().float().contiguous()
    _splitk(EPI_LN, x, w, y, bias=b, res=res, gamma=gamma, beta=beta, mean=mean, rstd=rstd, z=z, eps=eps,
            seed=seed, site=site, thr=thr, dscale=sc, row_map=row_map if thr else None,
            head=[hW, hb, labels, logits, dlogits, dz, colpart, hpart, dbpart, lpart, seed, loss.view(1),
                  _head_ticket(dev)],
            head_f=[float(head_site), float(hthr), float(hsc), float(kT), float(alpha), float(B)],
            head_dx=dx, head_tlogits=t, head_own=own)
    jobs.append((colpart, [dgamma, dbeta, dbias], M, 3 * N, N, acc_ln))
    jobs.append((hpart, [dW[0], dW[1]], M, 2 * N, N, acc_head))
    jobs.append((dbpart, [db[0:1], db[1:2]], M, 2, 1, acc_head))
    if loss_acc is not None:
        jobs.append((lpart, [loss_acc], M, 1, 1, True))
    return y, z, mean, rstd, (logits, loss, dz, dx if dx is not None else dz)


def linear_dx_ln_bwd(a, wt, res, z, gamma, mean, rstd, dgamma, dbeta, dbias, seed, site, p, accumulate=False,
                     row_map=None, jobs: Optional[list] = None, xsite=None, b_mn: bool = False, prefetch=None):
    """LayerNorm backward fused into the dX GEMM that produces its output gradient:
    dy = a wt^T + res, then (dz, dx) of y = LN(dropout(f) + r) from the saved z = dropout(f) + r
    (dz: gradient of the pre-LN sum, i.e. of the residual input r; dx: of f, = dz without dropout).
    dgamma / dbeta / dbias (+)= the column sums (deferred to ``colsum_flush`` with ``jobs``).
    b_mn=True: ``wt`` is the weight W [K, N] itself (dy = a W + res; no W^T copy needed)."""
    M, N = a.shape[0], (wt.shape[1] if b_mn else wt.shape[0])
    dz = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    thr, sc = _drop(p)
    dx = torch.empty_like(dz) if thr else None
    if _splitk_ok(M, N, a.shape[1]):
        key = "ln_colpart" if jobs is None else f"ln_colpart_job{len(jobs)}"
        ws = workspace(a.device, key, M * 3 * N)
        _splitk(EPI_LN_BWD, a, wt, dz, res=res, gamma=gamma, mean=mean, rstd=rstd, z=z, dx=dx, colpart=ws,
                seed=seed, site=site, thr=thr, dscale=sc, row_map=row_map if thr else None, b_mn=b_mn)
        job = (ws, [dgamma, dbeta, dbias], M, 3 * N, N, accumulate)
        if jobs is not None:
            jobs.append(job)
        else:
            colsum_flush([job])
        return dz, (dx if dx is not None else dz)
    key = "ln_colpart" if jobs is None else f"ln_colpart_job{len(jobs)}"
    ws = workspace(a.device, key, ((M + 63) // 64) * 3 * N)
    stats, cnt, err = _ln_state(a.device, M, N)
    xs = _xsite(a.device, N, xsite)
    nblk = ext().gemm_ln(True, a, wt, dz, None, res, gamma, None, mean, rstd, z, dx, ws, stats, cnt, err, 0.0, seed,
                         site, thr, sc, row_map if thr else None, LN_CFG, xs, b_mn, _ln2_xbuf(a.device),
                         _pf(prefetch))
    job = (ws, [dgamma, dbeta, dbias], nblk, 3 * N, N, accumulate)
    if jobs is not None:
        jobs.append(job)
    else:
        colsum_flush([job])
    return dz, (dx if dx is not None else dz)


def group_ids(ids: torch.Tensor):
    """(sorted ids, positions) grouping equal ids -- deterministic rank sort on device."""
    flat = ids.reshape(-1).contiguous()
    if flat.numel() > RANK_SORT_MAX:
        return torch.sort(flat, stable=True)
    srt = torch.empty(flat.numel(), dtype=torch.int64, device=flat.device)
    perm = torch.empty_like(srt)
    ext().rank_sort(flat, srt, perm)
    return srt, perm


RANK_SORT_MAX = 16384  # csrc/kernels/norm.hip rank sort: T ids in LDS


def emb_fwd(ids, word, pos, gamma, beta, S, eps, seed, site, p, row_map=None, ln_epoch=None, group=False,
            ln_stats=None):
    """row_map (int32 [T]): ``ids`` are packed real tokens; positions and dropout follow the padded row.
    ln_epoch (``ln_epoch(device)``): also advance the LayerNorm-fused GEMMs' exchange epoch;
    ln_stats (``ln_stats(device)``, with ln_epoch): the granules it zeroes when the tags wrap.
    group: also return the backward's id grouping (``group_ids``), computed by extra blocks of
    the same launch (T <= RANK_SORT_MAX; None beyond) -- the backward tail then has no sort launch."""
    T = ids.numel()
    D = gamma.numel()
    y = torch.empty(T, D, dtype=torch.bfloat16, device=ids.device)
    mean = torch.empty(T, dtype=torch.float32, device=ids.device)
    rstd = torch.empty(T, dtype=torch.float32, device=ids.device)
    thr, sc = _drop(p)
    srt = perm = None
    if group and T <= RANK_SORT_MAX:
        srt = torch.empty(T, dtype=torch.int64, device=ids.device)
        perm = torch.empty_like(srt)
    ext().emb_fwd(ids.contiguous(), word, pos, gamma, beta, y, mean, rstd, S, eps, seed, site, thr, sc, row_map,
                  ln_epoch, srt, perm, ln_stats)
    if group:
        return y, mean, rstd, ((srt, perm) if srt is not None else None)
    return y, mean, rstd


COLSUM_IN_EMB = _os.environ.get("FD_COLSUM_IN_EMB", "1") != "0"
COLSUM_JOBS_MAX = 32  # deferred column-sum jobs one launch takes (csrc/kernels/norm.hip COLSUM_MAXJ)


def emb_bwd(dy, ids, sorted_ids, perm, word, pos, gamma, mean, rstd, dword, dpos, dgamma, dbeta, S, seed, site, p,
            accumulate=False, now=None, ever=None, row_map=None, cu=None, colsum_jobs=None):
    """now/ever: optional uint8 [V] row flags -> sparse word gradient (see ArenaAdam).
    row_map / cu: packed rows (position gradient summed per sequence over cu).
    colsum_jobs: the backward's deferred column sums (``colsum_flush``'s list, <= COLSUM_JOBS_MAX):
    finalised by extra blocks of the embedding tail's first launch (the list is cleared)."""
    T = ids.numel()
    D = gamma.numel()
    dz = workspace(ids.device, "emb_dz", T * D)
    ws = workspace(ids.device, "emb_work", T * D + LN_GRID * 3 * D)  # word pieces, then LN partials
    thr, sc = _drop(p)
    jobs = colsum_jobs or []
    if len(jobs) > COLSUM_JOBS_MAX:
        raise ValueError(f"emb_bwd: {len(jobs)} column-sum jobs (<= {COLSUM_JOBS_MAX})")
    ext().emb_bwd(dy.contiguous(), ids.contiguous(), sorted_ids, perm, word, pos, gamma, mean, rstd, dword, dpos,
                  dgamma, dbeta, dz, ws, S, seed, site, thr, sc, accumulate, now, ever, row_map, cu,
                  [j[0] for j in jobs], [j[1] for j in jobs], [j[2] for j in jobs], [j[3] for j in jobs],
                  [j[4] for j in jobs], [int(j[5]) for j in jobs])
    if colsum_jobs:
        colsum_jobs.clear()


# ------------------------------------------------------------------ head / metrics / optimizer
def head_fwd(hidden, B, S, W, b, seed, site, p, labels=None, cls=None, kd=None, loss_acc=None):
    """cls (int32 [B]): packed layout -- sequence b's [CLS] is row cls[b] of hidden.
    kd = (teacher logits fp32 [B, 2], T, alpha): the fused loss is the distillation loss
    alpha * CE + (1 - alpha) * T^2 * KL(softmax(t/T) || softmax(z/T)) (models/bert.py kd_loss).
    loss_acc (fp32 [1], optional): the mean loss is also added to it on the device."""
    logits = torch.empty(B, 2, dtype=torch.float32, device=hidden.device)
    loss = dlogits = row_loss = None
    if labels is not None:
        loss = torch.empty((), dtype=torch.float32, device=hidden.device)
        dlogits = torch.empty(B, 2, dtype=torch.float32, device=hidden.device)
        row_loss = workspace(hidden.device, "head_row_loss", B)
    thr, sc = _drop(p)
    t, T, alpha = kd if kd is not None else (None, 1.0, 1.0)
    if t is not None:
        t = t.detach().float().contiguous()
    ext().head_fwd(hidden, B, S, W, b, seed, site, thr, sc, labels, logits, loss, dlogits, row_loss, cls,
                   t, float(T), float(alpha), loss_acc if labels is not None else None)
    return logits, loss, dlogits


def head_bwd(hidden, B, S, W, seed, site, p, dlogits, dW, db, accumulate=False, cls=None, gscale=None, own=None):
    """gscale: optional fp32 scalar tensor multiplying dlogits (a fused loss's upstream grad).
    own: packed sequence starts (int32 [B+1]); an empty sequence (own[b] == own[b+1]) gets no
    hidden-state gradient (its [CLS] row belongs to another sequence)."""
    dhidden = torch.empty_like(hidden)  # the kernel writes every row ([CLS] rows: gradient, others: 0)
    thr, sc = _drop(p)
    ext().head_bwd(hidden, B, S, W, seed, site, thr, sc, dlogits.contiguous(), dW, db, dhidden, accumulate, cls,
                   gscale, own)
    return dhidden


# The pruned training step's head forward + backward + output-LayerNorm backward as one launch
# (head_ln_bwd; FD_FUSE_HEAD=0: head_fwd, head_bwd and ln_bwd as three launches)
FUSE_HEAD = _os.environ.get("FD_FUSE_HEAD", "1") != "0"
_UNIT_GRAD = {}


def unit_grad(device) -> torch.Tensor:
    """The persistent fp32 scalar 1.0 a training step seeds ``loss.backward`` with (autograd would
    launch a fill per step).  A forward told ``unit_backward`` (the pruned step's fused head) has
    already applied the loss gradient for exactly this seed: its backward checks it got this tensor."""
    key = _dev_key(device)
    t = _UNIT_GRAD.get(key)
    if t is None:
        t = torch.ones((), dtype=torch.float32, device=device)
        _UNIT_GRAD[key] = t
    return t


def zero_scalar(device, dtype) -> torch.Tensor:
    """A persistent 0-d zero of ``dtype`` (expanded into a no-op gradient without a fill launch)."""
    key = (_dev_key(device), dtype)
    t = _UNIT_GRAD.get(key)
    if t is None:
        t = torch.zeros((), dtype=dtype, device=device)
        _UNIT_GRAD[key] = t
    return t


def head_ln_bwd(hidden, B, W, b, seed, head_site, p_head, labels, dW, db, acc_head, own, z, gamma, mean, rstd, site,
                p, row_map, dgamma, dbeta, dbias, acc_ln, jobs, kd=None, loss_acc=None):
    """The [CLS]-pruned training step's head in ONE launch (csrc/kernels/norm.hip
    head_ln_bwd_kernel), for a loss whose upstream gradient is 1: head forward (logits, loss mean,
    dlogits), head backward (dW / db (+)= ..., acc_head) and the last block's output-LayerNorm
    backward from the head gradient (z = its saved pre-LN sum [T, D], head row b = row b < B); the
    LN's dgamma / dbeta / dbias partials join the deferred column sums ``jobs``.  Bitwise the
    results of ``head_fwd`` + ``head_bwd`` + ``ln_bwd``.  Returns (logits, loss, dlogits, dz, dx)."""
    dev = hidden.device
    T, D = hidden.shape
    logits = torch.empty(B, 2, dtype=torch.float32, device=dev)
    loss = torch.empty((), dtype=torch.float32, device=dev)
    dlogits = torch.empty(B, 2, dtype=torch.float32, device=dev)
    row_loss = workspace(dev, "head_row_loss", B)
    hthr, hsc = _drop(p_head)
    thr, sc = _drop(p)
    t, kT, alpha = kd if kd is not None else (None, 1.0, 1.0)
    if t is not None:
        t = t.detach().float().contiguous()
    dz = torch.empty_like(z)
    dx = torch.empty_like(z) if thr else None
    ws = workspace(dev, f"ln_part_job{len(jobs)}", LN_BWD_PARTS * 3 * D)
    nblk = ext().head_ln_bwd(hidden, B, W, b, seed, head_site, hthr, hsc, labels, logits, loss, dlogits, row_loss,
                             loss_acc, dW, db, acc_head, own, t, float(kT), float(alpha), z, gamma, mean, rstd, dz,
                             dx, ws, site, thr, sc, row_map if thr else None)
    jobs.append((ws, [dgamma, dbeta, dbias], nblk, 3 * D, D, acc_ln))
    return logits, loss, dlogits, dz, (dx if dx is not None else dz)


def eval_metrics(logits, labels, acc, counts, prob1=None, preds=None):
    ext().eval_metrics(logits, labels, acc, counts, prob1, preds)


def adam(p, g, m, v, shadow, step, lr, b1, b2, eps, wd, decoupled, touched=None, now=None, skip_off=0, skip_rows=0,
         row_len=4, runs=None):
    """Flat-arena Adam.  touched/now (uint8 row flags over [skip_off, skip_off+skip_rows*row_len)) let
    the kernel skip rows with zero state and zero gradient (exact for weight_decay == 0).
    runs = (device int64 [n, 3] table, total float4s, largest end float4) from ``adam_runs``:
    update only those element runs, in one launch."""
    table, total4, end4 = runs if runs is not None else (None, 0, 0)
    ext().adam(p, g, m, v, shadow, step, lr, b1, b2, eps, wd, decoupled, touched, now, skip_off, skip_rows, row_len,
               table, total4, end4)


def adam_rows(p, g, m, v, shadow, step, lr, b1, b2, eps, ever, now, row_len):
    """Adam (weight decay 0) over the rows of one [rows][row_len] table (views of the arenas)
    whose ``ever`` flag is set -- the sparse word-embedding update, one wave per 64 row flags."""
    ext().adam_rows(p, g, m, v, shadow, step, lr, b1, b2, eps, ever, now, row_len)


def adam_runs(spans, device):
    """[(offset, numel)] element runs (multiples of 4, ascending, disjoint) -> the kernel's
    run table [start4, count4, prefix4] on ``device`` + its total and largest end (float4s)."""
    rows, pre, end = [], 0, 0
    for off, n in spans:
        if off % 4 or n % 4 or off < end:
            raise ValueError(f"adam run ({off}, {n}) not float4-aligned / ascending")
        rows.append((off // 4, n // 4, pre))
        pre += n // 4
        end = off + n
    return torch.tensor(rows, dtype=torch.int64, device=device), pre, end // 4


def step_inc(step=None, seed=None):
    ext().step_inc(step, seed)


def scale_cast(p, shadow=None, scale=1.0):
    ext().scale_cast(p, shadow, scale)


def axpby(dst, x, y=None, a=1.0, b=0.0):
    ext().axpby(dst, x, y, a, b)
