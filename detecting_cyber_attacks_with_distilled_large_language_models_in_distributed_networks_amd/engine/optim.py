"""Single-launch Adam / AdamW over the model's flat parameter arena.

Semantics = ``torch.optim.Adam(model.parameters(), lr=2e-5)`` of the reference
(client1.py:380: betas (0.9, 0.999), eps 1e-8, weight_decay 0, bias-corrected),
with an optional decoupled weight decay (AdamW; BASELINE.json says "AdamW
step" -- identical to Adam at wd = 0).

On GPU the update is the HIP Adam kernel (csrc/kernels/head_optim.hip), which
also refreshes the bf16 compute shadow; the step counter lives on the device so
the update can be replayed inside a HIP graph.  With ``overlap=True`` each
transformer block is updated on a side stream as soon as its
gradients are final, i.e. while the backward of the blocks below it still runs
(Adam is HBM-bound, the backward GEMMs are not), and ``step()`` only updates the
embeddings + head and joins the side stream.  (So between ``backward()`` and
``step()`` the blocks already hold their new weights; pass ``overlap=False`` for
gradient accumulation or to inspect weights there.)  On CPU the same math runs
as flat torch ops.

Measured on MI355X (bs32 x seq128): overlap makes the step SLOWER (3.86 vs
3.51 ms) -- the concurrent Adam blocks take CU slots from the one-round GEMM
grids and HBM bandwidth from LayerNorm/colsum -- so it is off by default.

Fused mode (``fuse_dw=True``, the default; active inside a training step's
``fused_adam_scope``): the encoder's 24 weight matrices (89 % of the dense
parameters) are updated by the weight-gradient GEMMs themselves -- the epilogue
applies Adam to the finished fp32 gradient tile (csrc/kernels/gemm.hip
``adam_epi4``, same arithmetic as the Adam kernel) instead of storing it, so the
gradient never round-trips through HBM and the p/m/v/shadow traffic streams
while other tiles of the grid are still on the MFMAs.  ``step()`` then updates
the rest (embeddings, biases, LayerNorms, head) in one launch over a run table.
The W^T copies the backward's dX GEMMs read are taken before the step, so a
block's later dX GEMMs still see the pre-update weights.  Bitwise identical to
the unfused step (tests/test_fused_adam_gpu.py, tests/test_dw_batch_gpu.py).

With the per-layer grouped dW launches (round 1) it did not pay: each grid runs as
one round, so every tile reached its Adam epilogue at the same time and the ~1.1 GB
of optimizer traffic overlapped nothing (2.39-2.42 vs 2.37-2.38 ms/step,
profiles/r1_ab_fused_adam_fixup.txt).  With all weight gradients of the step in ONE
launch at the end of the backward (RunCtx.dw_batch: ~20 rounds of tiles, no split-K)
the epilogues are staggered behind other tiles' MFMA work, and it does pay:
2.034-2.039 (batched, unfused) vs 1.999-2.000 ms/step (batched + fused), against
2.103 for the per-layer launches (profiles/r2_ab_dw_batch_fused_adam.txt).  On by
default; ``fuse_dw=False`` for the unfused arm.
"""
from __future__ import annotations

import math
from typing import Optional

import torch


class ArenaAdam:
    def __init__(self, model, lr: float = 2e-5, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, decoupled: bool = False, overlap: bool = False,
                 fuse_dw: bool = True):
        self.model = model
        self.overlap = overlap
        self.fuse_dw = fuse_dw
        self._run_tables = {}
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
        self._begun = False
        self._done = []  # (offset, length) spans already updated this step
        use = (self.overlap and dev.type == "cuda" and hasattr(self.model, "layer_span")
               and getattr(self.model, "impl", "hip") == "hip")
        self._side = torch.cuda.Stream(device=dev) if use else None
        if use:
            prev = self.model.layer_grads_hook
            if prev is not None and not isinstance(getattr(prev, "__self__", None), ArenaAdam):
                raise RuntimeError("ArenaAdam(overlap=True) cannot share the backward hook (data-parallel GradSync?)")
            self.model.layer_grads_hook = self._on_layer_grads

    def _begin(self, seed: Optional[torch.Tensor] = None, defer: Optional[list] = None):
        """Advance the device step counter once per step, before the first update launch.
        ``seed``: the model's dropout counter, advanced by the same launch (the model's training
        forward calls this inside a step scope: one tiny kernel instead of two).  ``defer``: append
        the (step, seed) counters to advance there instead of launching -- the caller folds them
        into a launch it makes anyway before anything reads them (the packing kernel)."""
        from ..ops import kernels as K
        if not self._begun:
            if defer is not None:
                defer.append((self.step_t, seed))
            else:
                K.step_inc(self.step_t, seed)
            self.host_step += 1
            self._begun = True
        elif seed is not None:
            if defer is not None:
                defer.append((None, seed))
            else:
                K.step_inc(None, seed)

    def _update(self, off: int, n: int, sparse: bool):
        from ..ops import kernels as K
        A = self.arena
        b1, b2 = self.betas
        sl = slice(off, off + n)
        if sparse:
            woff, rows, rl = self.model.word_embedding_span()
            K.adam(A.master[sl], A.grad[sl], self.m[sl], self.v[sl], A.shadow[sl], self.step_t, self.lr, b1, b2,
                   self.eps, self.weight_decay, self.decoupled, self.model.emb_ever, self.model.emb_now, woff - off,
                   rows, rl)
        else:
            K.adam(A.master[sl], A.grad[sl], self.m[sl], self.v[sl], A.shadow[sl], self.step_t, self.lr, b1, b2,
                   self.eps, self.weight_decay, self.decoupled)

    def _on_layer_grads(self, i: int):
        """Backward hook: block i's gradients are final -> update it on the side stream."""
        if not self.model.training or self._side is None:
            return
        self._begin()
        off, n = self.model.layer_span(i)
        if (off, n) in self._done:
            raise RuntimeError("block gradients finalised twice in one step (gradient accumulation needs "
                               "ArenaAdam(overlap=False))")
        cur = torch.cuda.current_stream(self.arena.device)
        self._side.wait_stream(cur)
        with torch.cuda.stream(self._side):
            self._update(off, n, False)
        self._done.append((off, n))

    def can_fuse(self) -> bool:
        """Whether the model's weight-gradient GEMMs may apply this optimizer's step."""
        m = self.model
        # the fused step updates weights inside the backward: safe only when every weight gradient
        # runs in the all-layer launch at the end (after the last dX GEMM that reads W)
        return (self.fuse_dw and not self.overlap and self.arena.device.type == "cuda"
                and getattr(m, "impl", "") == "hip" and getattr(m, "batch_dw", False)
                and getattr(m, "group_dw", False) and getattr(m, "layer_grads_hook", None) is None
                and self.arena.shadow is not None)

    def fused_args(self, grads):
        """(state tensors, hyper-parameters) for a weight-gradient GEMM that applies Adam to
        ``grads`` (arena grad views) in its epilogue; those spans are skipped by ``step()``."""
        from ..ops import kernels as K  # noqa: F401  (extension must be present)
        self._begin()
        A = self.arena
        base = A.grad.data_ptr()
        st = []
        for g in grads:
            off = (g.data_ptr() - base) // A.grad.element_size()
            n = g.numel()
            if not (0 <= off and off + n <= A.numel) or not g.is_contiguous():
                raise ValueError("fused Adam: gradient is not a contiguous arena view")
            st += [A.master[off:off + n], self.m[off:off + n], self.v[off:off + n], A.shadow[off:off + n]]
            self._done.append((off, n))
        st.append(self.step_t)
        b1, b2 = self.betas
        return st, [self.lr, b1, b2, self.eps, self.weight_decay, 1.0 if self.decoupled else 0.0]

    def _runs_table(self, runs):
        """Cached device run table for ``runs`` (built during the eager warm-up steps, so a
        graph capture never needs a host->device copy)."""
        key = tuple(runs)
        t = self._run_tables.get(key)
        if t is None:
            if torch.cuda.is_current_stream_capturing():
                return None
            from ..ops import kernels as K
            t = K.adam_runs(runs, self.arena.device)
            self._run_tables[key] = t
        return t

    def reset_state(self):
        """FedAvg rounds restart the moments (the reference re-creates Adam each run)."""
        self.m.zero_()
        self.v.zero_()
        self.step_t.zero_()
        self.host_step = 0
        self._done, self._begun = [], False
        self._rest_in_launch = False
        if getattr(self.model, "emb_ever", None) is not None:
            self.model.emb_ever.zero_()

    def zero_grad(self, set_to_none: bool = False):
        self.model.zero_grad()

    def mark_done(self, grads):
        """Arena gradient views that a launch other than ``step()`` updates this step (the qkv
        biases, updated by the all-layer weight-gradient tiles that sum their gradient)."""
        self._begin()
        A = self.arena
        base = A.grad.data_ptr()
        for g in grads:
            off = (g.data_ptr() - base) // A.grad.element_size()
            if not (0 <= off and off + g.numel() <= A.numel) or not g.is_contiguous():
                raise ValueError("mark_done: not a contiguous arena gradient view")
            self._done.append((off, g.numel()))

    def _sparse_words(self) -> bool:
        # Only the HIP path leaves a sparse word gradient (and sets the emb_now / emb_ever row
        # flags, in its embedding backward): the torch path's autograd writes the dense table
        # and sets no flag, so the row-flag Adam would skip every word row there.  (Round 3's
        # "HIP learns faster than fp32" loss-curve bias was exactly that: the fp32 reference
        # arm on the GPU never updated its word embeddings -- results/numerics_r4/.)
        hip_sparse = getattr(self.model, "impl", None) == "hip" and getattr(self.model, "sparse_word_grad", False)
        sparse = (hip_sparse and self.weight_decay == 0.0
                  and getattr(self.model, "emb_ever", None) is not None)
        if hip_sparse and not sparse and getattr(self.model, "emb_now", None) is not None:
            raise RuntimeError("sparse word-embedding grads need weight_decay == 0 "
                               "(set model.sparse_word_grad = False for AdamW)")
        return sparse

    def _rest_runs(self, sparse: bool):
        """(runs, rest): every element span not updated yet this step, and -- with the sparse word
        table -- the same minus that table (which the row-flag Adam takes)."""
        A = self.arena
        done = sorted(self._done)
        pos, runs = 0, []
        for off, n in done:
            if off > pos:
                runs.append((pos, off - pos))
            pos = max(pos, off + n)
        if pos < A.numel:
            runs.append((pos, A.numel - pos))
        if not sparse:
            return runs, None
        woff, rows, rl = self.model.word_embedding_span()
        wend = woff + rows * rl
        rest = []
        for off, n in runs:
            a, b = off, off + n
            if b <= woff or a >= wend:
                rest.append((a, n))
                continue
            if not (a <= woff and wend <= b):
                raise RuntimeError("the word-embedding table must lie inside one Adam run")
            if woff > a:
                rest.append((a, woff - a))
            if b > wend:
                rest.append((wend, b - wend))
        return runs, rest

    def rest_args(self):
        """The rest of this step's update for the all-layer weight-gradient launch to run beside its
        last tiles (csrc/kernels/gemm.hip dwb_rest; FD_ADAM_IN_DW=0: ``step()`` launches it):
        (tensors, ints) for ``gemm_dw_batch(rest=, rest_i=)``, or None when it cannot (no cached
        run table during a capture, a dense word table, ...).  Call after every other span of the
        step is marked done; ``step()`` then only finishes the bookkeeping."""
        from ..ops import kernels as K
        A = self.arena
        if not (K.ADAM_IN_DW and A.master.is_cuda and self._side is None and A.shadow is not None):
            return None
        self._begin()
        sparse = self._sparse_words()
        if not sparse:
            return None
        _, rest = self._rest_runs(True)
        if not rest:
            return None
        table = self._runs_table(rest)
        if table is None:
            return None
        woff, rows, rl = self.model.word_embedding_span()
        tab, total4, _ = table
        self._rest_in_launch = True
        return ([A.master, A.grad, self.m, self.v, A.shadow, tab, self.model.emb_ever, self.model.emb_now],
                [total4, woff, rows, rl])

    @torch.no_grad()
    def step(self):
        A = self.arena
        if A.master.device != self.m.device:
            self._alloc()
        b1, b2 = self.betas
        if A.master.is_cuda:
            self._begin()
            if getattr(self, "_rest_in_launch", False):
                # the all-layer weight-gradient launch already ran the rest (rest_args)
                self._rest_in_launch = False
                if self._side is not None:
                    torch.cuda.current_stream(A.device).wait_stream(self._side)
                self.model.mark_shadow_synced()
                self._done = []
                self._begun = False
                return
            sparse = self._sparse_words()
            # everything not already updated by the per-block hook, in contiguous runs
            runs, rest = self._rest_runs(sparse)
            woff = self.model.word_embedding_span()[0] if sparse else -1
            table = self._runs_table(runs) if len(runs) > 1 else None
            if table is not None and sparse:
                # the word-embedding table by its row flags (one wave per 64 rows: only rows with
                # Adam state are touched), everything else left in one run-table launch
                from ..ops import kernels as K
                _, rows, rl = self.model.word_embedding_span()
                wend = woff + rows * rl
                sl = slice(woff, wend)
                K.adam_rows(A.master[sl], A.grad[sl], self.m[sl], self.v[sl], A.shadow[sl], self.step_t, self.lr, b1,
                            b2, self.eps, self.model.emb_ever, self.model.emb_now, rl)
                rest_table = self._runs_table(rest) if len(rest) > 1 else None
                if rest_table is not None:
                    K.adam(A.master, A.grad, self.m, self.v, A.shadow, self.step_t, self.lr, b1, b2, self.eps,
                           self.weight_decay, self.decoupled, runs=rest_table)
                else:
                    for off, n in rest:
                        self._update(off, n, False)
            elif table is not None:  # everything left (fused-GEMM spans excluded) in one launch
                from ..ops import kernels as K
                b1, b2 = self.betas
                K.adam(A.master, A.grad, self.m, self.v, A.shadow, self.step_t, self.lr, b1, b2, self.eps,
                       self.weight_decay, self.decoupled, runs=table)
            else:
                for off, n in runs:
                    self._update(off, n, sparse and off <= woff < off + n)
            if self._side is not None:
                torch.cuda.current_stream(A.device).wait_stream(self._side)
            self.model.mark_shadow_synced()
            self._done = []
            self._begun = False
            return
        self.host_step += 1
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
