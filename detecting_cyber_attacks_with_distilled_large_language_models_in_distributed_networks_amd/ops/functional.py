"""Fused autograd blocks of the HIP DistilBERT path.

The model is three kinds of autograd nodes -- embeddings, one node per
TransformerBlock, and the classifier head -- each with a hand-ordered backward
that fuses across op boundaries (GELU-backward and residual-add in the dX GEMM
epilogues, dropout + residual + LayerNorm backward in one kernel, bias grads
out of the LN-backward column sums).  Parameter gradients are written straight
into the fp32 gradient arena (first write after ``zero_grad``, accumulate
otherwise), so autograd only ever carries activation gradients.

Reference call stack mirrored: DistilBertModel.forward -> Embeddings ->
6 x TransformerBlock -> [:, 0] -> Dropout(0.3) -> Linear(768, 2)
(client1.py:60-65).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Optional

import torch

from . import graph_split as _graph
from . import kernels as K


@dataclass
class RunCtx:
    """Per-forward shared state (one per model call)."""
    B: int
    S: int
    H: int
    kbias: torch.Tensor          # [B, S] additive key mask
    seed: torch.Tensor           # device int32 counter
    training: bool
    eps: float = 1e-12
    p_hidden: float = 0.1
    p_attn: float = 0.1
    p_head: float = 0.3
    # called with the layer index once a block's parameter gradients are final
    # (lets the optimizer update that block on a side stream during the rest of backward)
    on_layer_grads: Optional[Callable[[int], None]] = None
    # launch the weight gradients that become ready together (lin2 + lin1, out_lin + qkv)
    # as one grouped GEMM grid (fewer split-K slab round trips; csrc/kernels/gemm.hip)
    group_dw: bool = True
    # unpadded (packed) token layout: the transformer blocks run on the batch's real
    # tokens only.  cu = int32 [B+1] sequence starts (varlen attention), row_map = int32
    # [rows] packed -> padded row (-1 for the bucket's filler rows; dropout-hash index).
    cu: Optional[torch.Tensor] = None
    row_map: Optional[torch.Tensor] = None
    # packed layout at S > 128 whose every sequence has <= 128 tokens (the caller's
    # data.PackedTokens.max_len): varlen attention runs the S <= 128 kernels alone
    attn_short: bool = False
    # deferred column sums (bias / LN-affine grads): producers leave partials, the end of
    # the backward finalises all of them in one launch (None = finalise immediately)
    colsum_jobs: Optional[list] = None
    # deferred split-K weight-gradient reduces (ops/kernels.py dw_flush), same life cycle
    dw_jobs: Optional[list] = None
    # lin1's bias gradient from the GELU' dX GEMM's epilogue (needs colsum_jobs)
    fuse_colsum: bool = True
    # FFN activation g = gelu(u) not kept by the forward: the backward's GELU' dX GEMM re-creates
    # it next to its consumer (lin2's dW), so ~16.5 MB/layer less stays live across the step
    remat_gelu: bool = True
    # LayerNorm fused into the N = hidden GEMMs (csrc/kernels/gemm.hip gemm_ln_kernel): forward
    # out_lin + sa_layer_norm and lin2 + output_layer_norm; backward sa_layer_norm inside the
    # lin1 dX GEMM and block i-1's output_layer_norm inside block i's qkv dX GEMM
    fuse_ln: bool = False
    # the backward's LayerNorm-fused dX GEMMs (lin1 dX + sa_layer_norm, qkv dX + the previous
    # block's output_layer_norm); False while collectives run beside the backward (a data-parallel
    # client's overlapped gradient all-reduces: RCCL kernels hold CUs a row block's peers may
    # need -- ops/kernels.py ln_fusable) -> the plain dX GEMMs + separate LayerNorm backward
    fuse_ln_bwd: bool = True
    ln2_saved: dict = field(default_factory=dict)    # block -> its output LN's saved state
    ln2_pending: dict = field(default_factory=dict)  # block -> (dz2, df) computed by block + 1
    # optimizer whose Adam step the weight-gradient GEMMs apply in their epilogues
    # (engine/optim.py ArenaAdam.fused_args; set only inside a training step's scope)
    fused_adam: Optional[object] = None
    # all-layer weight gradients: the blocks only record (dy, x, grad, accumulate) and the
    # last backward node launches every weight gradient of the step as ONE grid
    # (ops/kernels.py linear_dw_batch; with ``fused_adam`` the Adam step runs in its epilogue)
    dw_batch: Optional[list] = None
    # with dw_batch + colsum_jobs: bf16 column sums whose source stays alive to the end of the
    # backward anyway (each block's dqkv, kept for the dW launch) -- their partials are computed
    # in ONE launch at the end (ops/kernels.py colsum_partials_batched) instead of one per block
    colsum_pending: Optional[list] = None
    # fp32 [1] device running sum of the fused loss (the model's ``loss_acc``): the head kernel
    # adds each step's mean loss, so a graph-replayed loop needs no add launch of its own
    loss_acc: Optional[torch.Tensor] = None
    # Last-block [CLS] pruning: the loss reads only each sequence's [CLS] row of the last block's
    # output, and every row of a block's FFN / out-proj / LayerNorms is computed independently of
    # the others, so in the LAST block only the [CLS] rows of everything after the attention can
    # reach the loss or any gradient (keys and values still need every row, so QKV and attention
    # run on all rows).  prune_idx = index of the pruned block (-1: off); cls_rows = int64 [Bp]
    # rows of the full layout to keep (the B [CLS] rows, then filler rows up to a multiple of 64 so
    # the pruned weight-gradient problems keep K % 64 == 0; their upstream gradient is 0);
    # cls_rmap = int32 [Bp] padded-row index of each kept row (dropout hash, same masks as the
    # unpruned path); head_rows = int32 [B] = arange(B) (the head reads the pruned output).
    prune_idx: int = -1
    cls_rows: Optional[torch.Tensor] = None
    cls_rmap: Optional[torch.Tensor] = None
    head_rows: Optional[torch.Tensor] = None
    # the caller seeds the loss's backward with ops/kernels.py unit_grad (engine/train.py): the
    # pruned step may then run the head's backward and the last block's output-LayerNorm backward
    # inside the forward's head launch (kernels.head_ln_bwd): pruned_ln2 = that LayerNorm's saved
    # state (from the pruned forward), head_fold = its (dz2, df) for the pruned block's backward
    unit_backward: bool = False
    pruned_ln2: Optional[tuple] = None
    head_fold: Optional[tuple] = None
    # the same fold one launch earlier (ops/kernels.py HEAD_IN_SK): head_req = (head handles,
    # labels, kd) set by the model before the blocks; the pruned block's output-LayerNorm split-K
    # epilogue then runs the head too and leaves head_done = (logits, loss, dz2, df) for HeadFn
    head_req: Optional[tuple] = None
    # every block's fused QKV weight, in block order (the forward's output-LN GEMM of block i prefetches
    # block i+1's: ops/kernels.py LN_PREFETCH)
    qkv_ws: Optional[list] = None
    head_done: Optional[tuple] = None


class GradSink:
    """Routes a parameter's gradient into its arena slice with first-write semantics."""

    def __init__(self, arena, name: str):
        self.arena, self.name = arena, name

    @property
    def buf(self) -> torch.Tensor:
        return self.arena.gview(self.name)

    def accumulate(self) -> bool:
        return self.arena.mark_written(self.name)

    def written(self) -> bool:
        """What ``accumulate`` would return, without marking the slot."""
        return self.arena.written(self.name)


class EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, token, ids, word, pos, gamma, beta, sinks, rc: RunCtx):
        p = rc.p_hidden if rc.training else 0.0
        # (the first launch of the forward also starts the fused LayerNorms' exchange epoch)
        # (a training forward's launch also groups the ids for the word gradient: no sort in the tail)
        group = bool(ctx.needs_input_grad[0])
        out = K.emb_fwd(ids, word, pos, gamma, beta, rc.S, rc.eps, rc.seed, 1, p, rc.row_map,
                        ln_epoch=K.ln_epoch(ids.device, gamma.numel()) if rc.fuse_ln else None, group=group,
                        ln_stats=K.ln_stats(ids.device, gamma.numel()) if rc.fuse_ln else None)
        y, mean, rstd = out[:3]
        ctx.grouped = out[3] if group else None
        ctx.rc, ctx.sinks, ctx.p = rc, sinks, p
        ctx.tensors = (ids, word, pos, gamma, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        EmbeddingFn._tail(ctx, dy)
        EmbeddingFn._weights(ctx.rc)
        return (None,) * 8

    @staticmethod
    def _weights(rc):
        if rc.dw_jobs:
            K.dw_flush(rc.dw_jobs)
        if rc.dw_batch:
            fa = rc.fused_adam
            acc_any = any(j[3] for j in rc.dw_batch)
            fused = fa is not None and not acc_any
            K.linear_dw_batch(rc.dw_batch, adam=fa.fused_args if fused else None, opt=fa if fused else None)
            rc.dw_batch.clear()

    @staticmethod
    def _tail(ctx, dy):
        ids, word, pos, gamma, mean, rstd = ctx.tensors
        s = ctx.sinks
        srt, perm = ctx.grouped if ctx.grouped is not None else K.group_ids(ids)
        acc = s["word"].accumulate()
        for k in ("pos", "ln_w", "ln_b"):
            assert s[k].accumulate() == acc
        now, ever = s.get("flags") or (None, None)
        rc = ctx.rc
        if rc.colsum_pending:
            K.colsum_partials_batched(rc.colsum_pending, rc.colsum_jobs)
        # the deferred column sums (every block's bias / LayerNorm-affine gradients) ride on the
        # embedding tail's first launch (FD_COLSUM_IN_EMB=0: a colsum_batched launch of their own)
        ride = rc.colsum_jobs if (K.COLSUM_IN_EMB and rc.colsum_jobs
                                  and len(rc.colsum_jobs) <= K.COLSUM_JOBS_MAX) else None
        K.emb_bwd(dy, ids, srt, perm, word, pos, gamma, mean, rstd, s["word"].buf, s["pos"].buf, s["ln_w"].buf,
                  s["ln_b"].buf, rc.S, rc.seed, 1, ctx.p, acc, now, ever, rc.row_map, rc.cu, colsum_jobs=ride)
        tt = s.get("type")
        if tt is not None:
            # BERT token-type row 0 is added at every position: d(type0) = sum_s d(pos_s).  The
            # position gradient already holds the running total of an accumulating backward,
            # so the type row is always re-derived from it (never added to) -- over EVERY
            # position row: an earlier micro-batch with a longer padded S accumulated into rows
            # this one does not reach (rows never reached are zero: pos_grad_kernel clears them)
            tt.accumulate()
            g = tt.buf
            torch.sum(s["pos"].buf, 0, out=g[0])
            g[1:].zero_()
        if ctx.rc.colsum_jobs:
            K.colsum_flush(ctx.rc.colsum_jobs)


class LayerFn(torch.autograd.Function):
    """One post-LN TransformerBlock: 7 kernels forward, 13 backward."""

    @staticmethod
    def forward(ctx, x, L, rc: RunCtx, idx: int):
        ctx.idx = idx
        ctx.pruned = idx == rc.prune_idx
        if ctx.pruned:
            return LayerFn._forward_pruned(ctx, x, L, rc, idx)
        p_a = rc.p_attn if rc.training else 0.0
        p_h = rc.p_hidden if rc.training else 0.0
        attn_site, ffn_site = 16 + 4 * idx, 17 + 4 * idx
        grad = ctx.needs_input_grad[0]
        sh = rc.attn_short
        dmask = K.attn_keep_bits(rc.B, rc.S, rc.H, p_a, x.device, short=sh) if grad else None
        if rc.fuse_ln and K.qkv_attn_ok(x.shape[0], x.shape[1], rc.S, short=sh):
            # QKV projection + attention in one launch (the exchange epoch advances per forward)
            qkv, cx, lse = K.qkv_attn_fwd(x, L["qkv_w"], L["qkv_b"], rc.kbias, rc.B, rc.S, rc.H, rc.seed, attn_site,
                                          p_a, rc.cu, dmask, xsite=K.ln_xsite(idx, 0, False), prefetch=L["o_w"],
                                          short=sh)
        else:
            qkv = K.linear_fwd(x, L["qkv_w"], L["qkv_b"], prefetch=L["o_w"])  # (out_lin follows attention)
            cx, lse = K.attn_fwd(qkv, rc.kbias, rc.B, rc.S, rc.H, rc.seed, attn_site, p_a, rc.cu, dmask,
                                 short=rc.attn_short)
        fuse_ln = rc.fuse_ln and K.ln_fusable(x.shape[0], x.shape[1], K=(x.shape[1], L["l2_w"].shape[1]))
        if fuse_ln:
            # bias + (dropout) + residual + LayerNorm in the N = 768 GEMMs' epilogues; the
            # backward reads the saved bf16 pre-LN sums z1 / z2 instead of ao / f
            # (each LayerNorm-fused GEMM touches the next launch's weight while it waits for its row
            # statistics: FFN1's, and the next block's QKV weight)
            nxt = rc.qkv_ws[idx + 1] if rc.qkv_ws is not None and idx + 1 < len(rc.qkv_ws) else None
            h, ao, m1, r1 = K.linear_ln_fwd(cx, L["o_w"], L["o_b"], x, L["ln1_w"], L["ln1_b"], rc.eps, rc.seed, 0,
                                            0.0, keep_z=grad, xsite=K.ln_xsite(idx, 0, False), prefetch=L["l1_w"])
            g, u = K.linear_fwd(h, L["l1_w"], L["l1_b"], gelu=True, prefetch=L["l2_w"], keep_u=grad)
            y, f, m2, r2 = K.linear_ln_fwd(g, L["l2_w"], L["l2_b"], h, L["ln2_w"], L["ln2_b"], rc.eps, rc.seed,
                                           ffn_site, p_h, rc.row_map, keep_z=grad, xsite=K.ln_xsite(idx, 1, False),
                                           prefetch=nxt)
            if grad:
                rc.ln2_saved[idx] = (f, m2, r2, L, ffn_site, p_h)
        else:
            ao = K.linear_fwd(cx, L["o_w"], L["o_b"])
            h, m1, r1 = K.ln_fwd(ao, x, L["ln1_w"], L["ln1_b"], rc.eps, rc.seed, 0, 0.0)
            g, u = K.linear_fwd(h, L["l1_w"], L["l1_b"], gelu=True, keep_u=grad)
            f = K.linear_fwd(g, L["l2_w"], L["l2_b"])
            y, m2, r2 = K.ln_fwd(f, h, L["ln2_w"], L["ln2_b"], rc.eps, rc.seed, ffn_site, p_h, rc.row_map)
        if grad:
            ctx.save_for_backward(x)
            # (fused LN: ao / f hold the pre-LN sums z1 / z2)
            ctx.acts = (qkv, cx, lse, ao, h, m1, r1, u, None if rc.remat_gelu else g, f, m2, r2)
            ctx.dmask = dmask
        ctx.L, ctx.rc, ctx.sites, ctx.p, ctx.fused_ln = L, rc, (attn_site, ffn_site), (p_a, p_h), fuse_ln
        _graph.split_point(idx)  # (a graph-chain boundary of a split training-step capture)
        return y

    @staticmethod
    def _forward_pruned(ctx, x, L, rc: RunCtx, idx: int):
        """The last block on its [CLS] rows only (RunCtx.prune_idx): QKV + attention on every row
        (keys / values), then out-proj + LN, FFN, LN on the gathered [CLS] rows.  Returns [Bp, D]."""
        p_a = rc.p_attn if rc.training else 0.0
        p_h = rc.p_hidden if rc.training else 0.0
        attn_site, ffn_site = 16 + 4 * idx, 17 + 4 * idx
        grad = ctx.needs_input_grad[0]
        sh = rc.attn_short
        dmask = K.attn_keep_bits(rc.B, rc.S, rc.H, p_a, x.device, short=sh) if grad else None
        # only each sequence's first query row ([CLS]) is needed: the other rows' context is never read
        ci, rm = rc.cls_rows, rc.cls_rmap
        if rc.fuse_ln and K.attn_cls_compact_ok(rc.S, sh) and K.qkv_attn_ok(x.shape[0], x.shape[1], rc.S, short=sh):
            # QKV projection + [CLS]-row attention (+ the compact rows) in one launch
            qkv, cx, lse, cxc, xc = K.qkv_attn_fwd(x, L["qkv_w"], L["qkv_b"], rc.kbias, rc.B, rc.S, rc.H, rc.seed,
                                                   attn_site, p_a, rc.cu, dmask, q_live=1, cls=(x, ci.numel()),
                                                   xsite=K.ln_xsite(idx, 0, False), short=sh)
        elif K.attn_cls_compact_ok(rc.S, sh):  # the attention launch also writes the compact [CLS] rows
            qkv = K.linear_fwd(x, L["qkv_w"], L["qkv_b"])
            cx, lse, cxc, xc = K.attn_fwd(qkv, rc.kbias, rc.B, rc.S, rc.H, rc.seed, attn_site, p_a, rc.cu, dmask,
                                          q_live=1, cls=(x, ci.numel()), short=sh)
        else:
            qkv = K.linear_fwd(x, L["qkv_w"], L["qkv_b"])
            cx, lse = K.attn_fwd(qkv, rc.kbias, rc.B, rc.S, rc.H, rc.seed, attn_site, p_a, rc.cu, dmask, q_live=1,
                                 short=rc.attn_short)
            cxc, xc = K.gather_rows2(cx, x, ci)
        h, ao, m1, r1 = K.linear_ln_fwd(cxc, L["o_w"], L["o_b"], xc, L["ln1_w"], L["ln1_b"], rc.eps, rc.seed, 0, 0.0,
                                        keep_z=grad, xsite=K.ln_xsite(idx, 0, False))
        g, u = K.linear_fwd(h, L["l1_w"], L["l1_b"], gelu=True, keep_u=grad)
        hq = rc.head_req if grad else None
        if hq is not None and K.head_in_sk_ok(g.shape[0], L["l2_w"].shape[0], g.shape[1]):
            # the head + this LayerNorm's backward in the LayerNorm's own split-K epilogue launch
            head, labels, kd = hq
            G = L["sinks"]
            hs = head["sinks"]
            acc_ln = G["l2_w"].written()  # (peek: the pruned block's backward marks it)
            acc_h = hs["w"].accumulate()
            hs["b"].accumulate()
            y, f, m2, r2, hout = K.linear_ln_fwd_head(
                g, L["l2_w"], L["l2_b"], h, L["ln2_w"], L["ln2_b"], rc.eps, rc.seed, ffn_site, p_h, rm,
                head["w"], head["b"], 2, rc.p_head, labels, rc.B, rc.cu, kd, hs["w"].buf, hs["b"].buf, acc_h,
                G["ln2_w"].buf, G["ln2_b"].buf, G["l2_b"].buf, acc_ln, rc.colsum_jobs, rc.loss_acc)
            rc.head_done = hout
            rc.head_req = None
        else:
            y, f, m2, r2 = K.linear_ln_fwd(g, L["l2_w"], L["l2_b"], h, L["ln2_w"], L["ln2_b"], rc.eps, rc.seed,
                                           ffn_site, p_h, rm, keep_z=grad, xsite=K.ln_xsite(idx, 1, False))
        if grad:
            ctx.save_for_backward(x)
            ctx.acts = (qkv, cx, lse, cxc, ao, h, m1, r1, u, None if rc.remat_gelu else g, f, m2, r2)
            ctx.dmask = dmask
            rc.pruned_ln2 = (f, m2, r2, L, ffn_site, p_h, rm)
        ctx.L, ctx.rc, ctx.sites, ctx.p = L, rc, (attn_site, ffn_site), (p_a, p_h)
        return y

    @staticmethod
    def _backward_pruned(ctx, dy):
        """Backward of _forward_pruned: LayerNorm / FFN / out-proj on the Bp kept rows (their
        weight gradients join the all-layer dW launch with K = Bp), the attention backward and the
        QKV dX on every row with the [CLS] gradients scattered back (other rows' are exactly 0)."""
        (x,) = ctx.saved_tensors
        qkv, cx, lse, cxc, ao, h, m1, r1, u, g, f, m2, r2 = ctx.acts
        L, rc = ctx.L, ctx.rc
        G = L["sinks"]
        attn_site, ffn_site = ctx.sites
        p_a, p_h = ctx.p
        acc = G["l2_w"].accumulate()
        jobs = rc.colsum_jobs
        batch = rc.dw_batch
        ci, rm, B = rc.cls_rows, rc.cls_rmap, rc.B
        if rc.head_fold is not None:
            dz2, df = rc.head_fold  # the output-LayerNorm backward ran in the head's launch (HeadFn)
            rc.head_fold = None
        else:
            dz2, df = K.ln_bwd(dy, f, None, L["ln2_w"], m2, r2, G["ln2_w"].buf, G["ln2_b"].buf, G["l2_b"].buf, rc.seed,
                               ffn_site, p_h, acc, rm, jobs, zin=True)
        g_out = torch.empty_like(u) if g is None else None
        fuse_cs = jobs is not None and rc.fuse_colsum
        du = K.linear_dx(df, L["l2_w"], gelu_u=u,
                         colsum=(jobs, G["l1_b"].buf, acc) if fuse_cs else None, aux_out=g_out)
        if not fuse_cs:
            K.colsum(du, G["l1_b"].buf, acc, jobs)
        if g is None:
            g = g_out
        batch += [(df, g, G["l2_w"].buf, acc), (du, h, G["l1_w"].buf, acc)]
        dz1c, _ = K.linear_dx_ln_bwd(du, L["l1_w"], dz2, ao, L["ln1_w"], m1, r1, G["ln1_w"].buf, G["ln1_b"].buf,
                                     G["o_b"].buf, rc.seed, 0, 0.0, acc, None, jobs, xsite=K.ln_xsite(ctx.idx, 0, True),
                                     b_mn=True, prefetch=L["o_w"])
        sh = rc.attn_short
        if K.attn_cls_compact_ok(rc.S, sh) and K.attn_bwd_proj_ok(rc.S, cls=True, short=sh):
            # the out-projection's dX of the [CLS] rows inside the attention backward, which also
            # scatters dz1c into the full layout
            dqkv, dz1 = K.attn_bwd_proj(qkv, rc.kbias, cx, lse, dz1c, L["o_w"], rc.B, rc.S, rc.H, rc.seed, attn_site,
                                        p_a, rc.cu, ctx.dmask, dresc=dz1c, short=sh)
        elif K.attn_cls_compact_ok(rc.S, sh):
            dcxc = K.linear_dx(dz1c, L["o_w"])
            # the attention backward reads the compact [CLS] gradient and scatters dz1c into the
            # full layout itself (every other row exactly 0)
            dqkv, dz1 = K.attn_bwd(qkv, rc.kbias, cx, lse, dcxc, rc.B, rc.S, rc.H, rc.seed, attn_site, p_a, rc.cu,
                                   ctx.dmask, q_live=1, dresc=dz1c, short=sh)
        else:
            dcxc = K.linear_dx(dz1c, L["o_w"])
            # the [CLS] rows' gradients back into the full layout (every other row exactly 0)
            dcx, dz1 = K.scatter_rows2(dcxc, dz1c, ci, B, cx.shape[0])
            dqkv = K.attn_bwd(qkv, rc.kbias, cx, lse, dcx, rc.B, rc.S, rc.H, rc.seed, attn_site, p_a, rc.cu,
                              ctx.dmask, q_live=1, short=rc.attn_short)
        # (the qkv bias gradient: column sums of dqkv in the dW launch's qkv tiles, K.DW_QKV_BIAS)
        batch += [(dz1c, cxc, G["o_w"].buf, acc),
                  (dqkv, x, G["qkv_w"].buf, acc, G["qkv_b"].buf if K.DW_QKV_BIAS else None)]
        if not K.DW_QKV_BIAS:
            if rc.colsum_pending is not None:
                rc.colsum_pending.append((dqkv, G["qkv_b"].buf, acc))
            else:
                K.colsum(dqkv, G["qkv_b"].buf, acc, jobs)
        prev = rc.ln2_saved.get(ctx.idx - 1) if rc.fuse_ln_bwd else None
        if prev is not None:
            z2p, m2p, r2p, Lp, site_p, p_p = prev
            Gp = Lp["sinks"]
            acc_p = [Gp[k].accumulate() for k in ("ln2_w", "ln2_b", "l2_b")]
            if len(set(acc_p)) != 1:
                raise RuntimeError("output-LN gradient sinks out of step")
            dx, df_p = K.linear_dx_ln_bwd(dqkv, L["qkv_w"], dz1, z2p, Lp["ln2_w"], m2p, r2p, Gp["ln2_w"].buf,
                                          Gp["ln2_b"].buf, Gp["l2_b"].buf, rc.seed, site_p, p_p, acc_p[0], rc.row_map,
                                          jobs, xsite=K.ln_xsite(ctx.idx, 1, True), b_mn=True,
                                          prefetch=Lp["l2_w"])
            rc.ln2_pending[ctx.idx - 1] = (dx, df_p)
        else:
            dx = K.linear_dx(dqkv, L["qkv_w"], res=dz1)
        for k in ("qkv_w", "qkv_b", "o_w", "o_b", "ln1_w", "ln1_b", "l1_w", "l1_b", "l2_b", "ln2_w", "ln2_b"):
            G[k].accumulate()
        del ctx.acts, ctx.dmask
        return dx, None, None, None

    @staticmethod
    def backward(ctx, dy):
        if ctx.pruned:
            return LayerFn._backward_pruned(ctx, dy)
        (x,) = ctx.saved_tensors
        qkv, cx, lse, ao, h, m1, r1, u, g, f, m2, r2 = ctx.acts
        L, rc = ctx.L, ctx.rc
        G = L["sinks"]
        attn_site, ffn_site = ctx.sites
        p_a, p_h = ctx.p
        acc = G["l2_w"].accumulate()
        # output_layer_norm(dropout(lin2) + h): dz2 -> residual grad of h, df -> lin2 output grad
        jobs = rc.colsum_jobs
        fused = ctx.fused_ln
        fused_bwd = fused and rc.fuse_ln_bwd
        pend = rc.ln2_pending.pop(ctx.idx, None) if fused else None
        if pend is not None and pend[0].data_ptr() == dy.data_ptr():
            dz2, df = pend  # done by block idx + 1's qkv dX GEMM (its returned "dx" IS dz2)
        else:
            # fused forward: f holds z2 (the pre-LN sum), the residual is already in it
            dz2, df = K.ln_bwd(dy, f, None if fused else h, L["ln2_w"], m2, r2, G["ln2_w"].buf, G["ln2_b"].buf,
                               G["l2_b"].buf, rc.seed, ffn_site, p_h, acc, rc.row_map, jobs, zin=fused)
        batch = rc.dw_batch  # all-layer weight gradients: record now, one launch at the end
        # dg W2 * gelu'(u); with deferred column sums the epilogue also leaves lin1's bias-gradient
        # partials (no separate pass over du)
        fuse_cs = jobs is not None and rc.fuse_colsum
        g_out = torch.empty_like(u) if g is None else None  # re-created gelu(u) (RunCtx.remat_gelu)
        du = K.linear_dx(df, L["l2_w"], gelu_u=u,
                         colsum=(jobs, G["l1_b"].buf, acc) if fuse_cs else None, aux_out=g_out,
                         prefetch=L["l1_w"])
        if g is None:
            g = g_out
        if batch is not None:
            batch += [(df, g, G["l2_w"].buf, acc), (du, h, G["l1_w"].buf, acc)]
        elif rc.group_dw:
            # (the per-block weight gradients run while later dX GEMMs still read W: no fused Adam)
            K.linear_dw2(df, g, G["l2_w"].buf, du, h, G["l1_w"].buf, acc, jobs=rc.dw_jobs)
        else:
            K.linear_dw(df, g, G["l2_w"].buf, acc)
            K.linear_dw(du, h, G["l1_w"].buf, acc)
        if not fuse_cs:
            K.colsum(du, G["l1_b"].buf, acc, jobs)
        # sa_layer_norm(out_lin + x): dh = du W1 + dz2, then its LayerNorm backward
        if fused_bwd:
            dz1, _ = K.linear_dx_ln_bwd(du, L["l1_w"], dz2, ao, L["ln1_w"], m1, r1, G["ln1_w"].buf, G["ln1_b"].buf,
                                        G["o_b"].buf, rc.seed, 0, 0.0, acc, None, jobs,
                                        xsite=K.ln_xsite(ctx.idx, 0, True), b_mn=True, prefetch=L["o_w"])
        else:
            dh = K.linear_dx(du, L["l1_w"], res=dz2)
            dz1, _ = K.ln_bwd(dh, ao, None if fused else x, L["ln1_w"], m1, r1, G["ln1_w"].buf, G["ln1_b"].buf,
                              G["o_b"].buf, rc.seed, 0, 0.0, acc, None, jobs, zin=fused)
        if not rc.group_dw and batch is None:
            K.linear_dw(dz1, cx, G["o_w"].buf, acc)
        if K.attn_bwd_proj_ok(rc.S, short=rc.attn_short):  # the out-projection's dX inside the attention backward
            dqkv = K.attn_bwd_proj(qkv, rc.kbias, cx, lse, dz1, L["o_w"], rc.B, rc.S, rc.H, rc.seed, attn_site, p_a,
                                   rc.cu, ctx.dmask, short=rc.attn_short)
        else:
            dcx = K.linear_dx(dz1, L["o_w"])
            dqkv = K.attn_bwd(qkv, rc.kbias, cx, lse, dcx, rc.B, rc.S, rc.H, rc.seed, attn_site, p_a, rc.cu,
                              ctx.dmask, short=rc.attn_short)
        dw_bias = batch is not None and K.DW_QKV_BIAS  # qkv bias gradient in the dW launch
        if batch is not None:
            batch += [(dz1, cx, G["o_w"].buf, acc),
                      (dqkv, x, G["qkv_w"].buf, acc, G["qkv_b"].buf if dw_bias else None)]
        elif rc.group_dw:
            K.linear_dw2(dz1, cx, G["o_w"].buf, dqkv, x, G["qkv_w"].buf, acc, jobs=rc.dw_jobs)
        else:
            K.linear_dw(dqkv, x, G["qkv_w"].buf, acc)
        if not dw_bias:
            if batch is not None and jobs is not None and rc.colsum_pending is not None:
                rc.colsum_pending.append((dqkv, G["qkv_b"].buf, acc))  # partials at the end, batched
            else:
                K.colsum(dqkv, G["qkv_b"].buf, acc, jobs)
        prev = rc.ln2_saved.get(ctx.idx - 1) if fused_bwd else None
        if prev is not None:
            # dx = dqkv Wqkv + dz1 is block idx-1's output-LN gradient: finish that LayerNorm
            # backward in this GEMM's epilogue and hand (dz2, df) to block idx-1
            z2p, m2p, r2p, Lp, site_p, p_p = prev
            Gp = Lp["sinks"]
            acc_p = [Gp[k].accumulate() for k in ("ln2_w", "ln2_b", "l2_b")]
            if len(set(acc_p)) != 1:
                raise RuntimeError("output-LN gradient sinks out of step")
            acc_p = acc_p[0]
            dx, df_p = K.linear_dx_ln_bwd(dqkv, L["qkv_w"], dz1, z2p, Lp["ln2_w"], m2p, r2p, Gp["ln2_w"].buf,
                                          Gp["ln2_b"].buf, Gp["l2_b"].buf, rc.seed, site_p, p_p, acc_p, rc.row_map,
                                          jobs, xsite=K.ln_xsite(ctx.idx, 1, True), b_mn=True,
                                          prefetch=Lp["l2_w"])
            rc.ln2_pending[ctx.idx - 1] = (dx, df_p)
        else:
            dx = K.linear_dx(dqkv, L["qkv_w"], res=dz1)
        for k in ("qkv_w", "qkv_b", "o_w", "o_b", "ln1_w", "ln1_b", "l1_w", "l1_b", "l2_b", "ln2_w", "ln2_b"):
            G[k].accumulate()
        del ctx.acts, ctx.dmask
        if rc.on_layer_grads is not None:
            rc.on_layer_grads(ctx.idx)  # (stream-ordered after this block's dW work and LN grads)
        return dx, None, None, None


class HeadFn(torch.autograd.Function):
    """CLS -> Dropout(0.3) -> Linear(768, 2); optional fused CE (mean) loss."""

    @staticmethod
    def forward(ctx, hidden, W, b, sinks, rc: RunCtx, labels: Optional[torch.Tensor], kd=None):
        """kd = (teacher logits, T, alpha): the fused loss is the distillation loss."""
        p = rc.p_head if rc.training else 0.0
        ctx.rc, ctx.sinks, ctx.p, ctx.W = rc, sinks, p, W
        ctx.fused_loss = labels is not None
        ctx.folded = False
        hd = rc.head_done
        if hd is not None and labels is not None and ctx.needs_input_grad[0]:
            # the pruned block's output-LayerNorm launch already ran the head (forward and backward)
            logits, loss, dz2, df = hd
            rc.head_done = None
            rc.head_fold = (dz2, df)
            rc.pruned_ln2 = None
            ctx.folded = True
            ctx.unit = K.unit_grad(hidden.device)
            ctx.zero = K.zero_scalar(hidden.device, hidden.dtype)
            ctx.shape = hidden.shape
            ctx.set_materialize_grads(False)
            ctx.mark_non_differentiable(logits)
            return loss, logits
        ln2 = rc.pruned_ln2
        if (K.FUSE_HEAD and labels is not None and rc.training and rc.unit_backward and ctx.needs_input_grad[0]
                and ln2 is not None and rc.head_rows is not None and rc.colsum_jobs is not None
                and hidden.shape[0] == ln2[0].shape[0] and hidden.shape[1] == 768):
            # pruned step, loss seeded with unit_grad: head forward + backward + the last block's
            # output-LayerNorm backward in this one launch (the backward nodes only pick it up)
            f, m2, r2, L, ffn_site, p_h, rm = ln2
            G = L["sinks"]
            acc_ln = G["l2_w"].written()  # (peek: the pruned block's backward marks it)
            acc_h = sinks["w"].accumulate()
            sinks["b"].accumulate()
            logits, loss, dlog, dz2, df = K.head_ln_bwd(
                hidden, rc.B, W, b, rc.seed, 2, p, labels, sinks["w"].buf, sinks["b"].buf, acc_h, rc.cu, f,
                L["ln2_w"], m2, r2, ffn_site, p_h, rm, G["ln2_w"].buf, G["ln2_b"].buf, G["l2_b"].buf, acc_ln,
                rc.colsum_jobs, kd=kd, loss_acc=rc.loss_acc)
            rc.head_fold = (dz2, df)
            rc.pruned_ln2 = None
            ctx.folded = True
            ctx.unit = K.unit_grad(hidden.device)
            ctx.zero = K.zero_scalar(hidden.device, hidden.dtype)
            ctx.shape = hidden.shape
            ctx.set_materialize_grads(False)
            ctx.mark_non_differentiable(logits)
            return loss, logits
        # packed: [CLS] = first row of each sequence; pruned last block: row b of its output
        cls = rc.head_rows if rc.head_rows is not None else rc.cu[:-1] if rc.cu is not None else None
        logits, loss, dlog = K.head_fwd(hidden, rc.B, rc.S, W, b, rc.seed, 2, p, labels, cls, kd,
                                        loss_acc=rc.loss_acc if rc.training else None)
        ctx.save_for_backward(hidden)
        ctx.dlog = dlog
        ctx.set_materialize_grads(False)  # the unused output's grad stays None (no fill launch)
        if labels is not None:
            ctx.mark_non_differentiable(logits)  # the gradient flows through the fused loss
            return loss, logits
        dummy = logits.new_empty(0)
        ctx.mark_non_differentiable(dummy)
        return logits, dummy

    @staticmethod
    def backward(ctx, g0, g1):
        if ctx.folded:
            # the forward's launch already applied this gradient (for a seed of exactly unit_grad)
            if g0 is not None and g0.data_ptr() != ctx.unit.data_ptr():
                raise RuntimeError("the fused pruned head expects loss.backward(ops.kernels.unit_grad(device)) "
                                   "(forward_loss(..., unit_backward=True) promised it)")
            return (ctx.zero.expand(ctx.shape),) + (None,) * 6
        (hidden,) = ctx.saved_tensors
        gscale = None
        if ctx.fused_loss:
            if g0 is None:
                return (None,) * 7
            dlog = ctx.dlog
            gscale = g0.float().reshape(1)  # scaled inside the kernel (no elementwise launch)
        else:
            if g0 is None:
                return (None,) * 7
            dlog = g0.float().contiguous()
        s = ctx.sinks
        acc = s["w"].accumulate()
        s["b"].accumulate()
        rc = ctx.rc
        cls = rc.head_rows if rc.head_rows is not None else rc.cu[:-1] if rc.cu is not None else None
        dh = K.head_bwd(hidden, ctx.rc.B, ctx.rc.S, ctx.W, ctx.rc.seed, 2, ctx.p, dlog, s["w"].buf, s["b"].buf, acc,
                        cls, gscale, own=rc.cu)
        return dh, None, None, None, None, None, None
