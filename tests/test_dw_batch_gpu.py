"""All-layer weight gradients in one launch (csrc/kernels/gemm.hip gemm_dw_batch_kernel).

* kernel: every problem of a batch == the fp32 product dy^T x (accumulate too), for the
  DistilBERT shapes of a packed bs32 step and for several tile configurations;
* model: the batched backward gives the per-layer (grouped, split-K) gradients up to fp32
  summation order, and Adam fused into the batched epilogue reproduces gradient-then-Adam bit
  for bit (training steps, eager and graph-replayed).
"""
import pytest
import torch

from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.engine import (
    ArenaAdam, GraphedTrainStep, make_step_fn)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.models import (
    DDoSClassifier, DistilBertConfig)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K

pytestmark = pytest.mark.gpu


def _frel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("cfg", [-1, 1, 8, 11])
def test_dw_batch_kernel_matches_fp32(cfg):
    g = torch.Generator(device="cuda").manual_seed(cfg + 5)
    T = 2688
    shapes = [(768, 3072), (3072, 768), (768, 768), (2304, 768)] * 2
    jobs, refs = [], []
    for i, (M, N) in enumerate(shapes):
        dy = (torch.randn(T, M, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
        x = torch.randn(T, N, device="cuda", generator=g).to(torch.bfloat16)
        acc = i % 3 == 2
        out = torch.randn(M, N, device="cuda", generator=g) if acc else torch.empty(M, N, device="cuda")
        ref = dy.float().t() @ x.float() + (out.clone() if acc else 0.0)
        jobs.append((dy, x, out, acc))
        refs.append(ref)
    K.linear_dw_batch(jobs, cfg=cfg)
    torch.cuda.synchronize()
    for (_, _, out, _), ref in zip(jobs, refs):
        assert _frel(out, ref) < 1e-5, _frel(out, ref)


def _batch(B, S, seed=0):
    gen = torch.Generator().manual_seed(seed)
    ids = torch.randint(1000, 2000, (B, S), generator=gen)
    lens = torch.randint(S // 3, S + 1, (B,), generator=gen)
    mask = (torch.arange(S)[None] < lens[:, None]).long()
    ids = ids * mask
    ids[:, 0] = 101
    labels = torch.randint(0, 2, (B,), generator=gen)
    return ids.cuda(), mask.cuda(), labels.cuda(), int(lens.sum())


def test_batched_backward_matches_per_layer():
    cfg = DistilBertConfig(n_layers=3)
    grads = []
    for batch in (True, False):
        m = DDoSClassifier(config=cfg, device="cuda", impl="hip", seed=17)
        m.batch_dw = batch
        m.prune_last = False  # (pruning needs the batched launch; it is compared in test_prune_gpu.py)
        m.train()
        ids, mask, labels, tokens = _batch(32, 128, seed=400)
        for acc_step in range(2):  # the second backward accumulates into the gradients
            if acc_step == 0:
                m.zero_grad()
            m.rng.fill_(acc_step)
            loss, _ = m.forward_loss(ids, mask, labels, tokens=tokens)
            loss.backward()
        torch.cuda.synchronize()
        grads.append({k: m.dense_grad(k).clone() for k in m.state_dict()})
    for k in grads[0]:
        if grads[1][k].norm() > 0:
            assert _frel(grads[0][k], grads[1][k]) < 1e-4, k


@pytest.mark.parametrize("graph", [False, True])
def test_fused_adam_in_batched_dw_matches_unfused(graph):
    cfg = DistilBertConfig(n_layers=2)
    models, opts, steps = [], [], []
    for fuse in (True, False):
        m = DDoSClassifier(config=cfg, device="cuda", impl="hip", seed=19)
        m.batch_dw = True
        m.train()
        opt = ArenaAdam(m, lr=1e-3, fuse_dw=fuse)
        assert opt.can_fuse() == fuse
        models.append(m)
        opts.append(opt)
        steps.append(GraphedTrainStep(make_step_fn(m, opt), warmup=1, enabled=graph, bucket=m.packed_rows))
    for it in range(5):
        ids, mask, labels, tokens = _batch(16, 128, seed=500 + it)
        for st in steps:
            st(ids, mask, labels, tokens)
    torch.cuda.synchronize()
    a, b = models[0].arena, models[1].arena
    assert opts[0]._done == []
    assert torch.equal(a.master, b.master)
    assert torch.equal(opts[0].m, opts[1].m) and torch.equal(opts[0].v, opts[1].v)
    assert torch.equal(a.shadow, b.shadow)
    if graph:
        assert all(st.graph is not None and st.failed is None for st in steps)


def test_batched_qkv_bias_partials_bitwise():
    """The per-block qkv-bias column-sum partials computed in one launch at the end of the
    backward (model.batch_colsum, ops/kernels.py colsum_partials_batched) give bitwise the
    gradients of one partial launch per block -- including an accumulating second backward."""
    cfg = DistilBertConfig(n_layers=3)
    grads = []
    for batched in (True, False):
        m = DDoSClassifier(config=cfg, device="cuda", impl="hip", seed=29)
        m.batch_colsum = batched
        m.train()
        ids, mask, labels, tokens = _batch(32, 128, seed=700)
        for acc_step in range(2):
            if acc_step == 0:
                m.zero_grad()
            m.rng.fill_(acc_step)
            loss, _ = m.forward_loss(ids, mask, labels, tokens=tokens)
            loss.backward()
        torch.cuda.synchronize()
        grads.append(m.arena.grad.clone())
    assert torch.equal(grads[0], grads[1])


def test_colsum_partials_batched_kernel():
    g = torch.Generator(device="cuda").manual_seed(3)
    xs = [torch.randn(T, N, device="cuda", generator=g).to(torch.bfloat16) for T, N in ((2688, 2304), (700, 768), (33, 3072))]
    outs_a = [torch.zeros(x.shape[1], device="cuda") for x in xs]
    outs_b = [torch.ones(x.shape[1], device="cuda") for x in xs]
    jobs_a, jobs_b = [], []
    for x, o in zip(xs, outs_a):
        K.colsum(x, o, False, jobs_a)
    K.colsum_flush(jobs_a)
    K.colsum_partials_batched([(x, o, True) for x, o in zip(xs, outs_b)], jobs_b)
    K.colsum_flush(jobs_b)
    torch.cuda.synchronize()
    for x, a, b in zip(xs, outs_a, outs_b):
        assert torch.equal(a + 1.0, b)
        assert ((a - x.float().sum(0)).abs().max() / x.float().sum(0).abs().max()).item() < 1e-5


def test_dw_tail_launch_bitwise_equals_single_launch():
    """FD_DW_TAIL: the last, mostly empty round of 256 x 256 tiles (and the pruned block's short-K
    problems) goes to a second launch of 128 x 128 tiles.  Every output element accumulates the
    same K products in the same order and takes the same fused Adam step: bitwise equal."""
    g = torch.Generator(device="cuda").manual_seed(9)
    T, Tc = 2688, 64
    shapes = [(2304, 768, T), (768, 768, T), (3072, 768, T), (768, 3072, T)] * 5 + \
        [(2304, 768, T), (768, 768, Tc), (3072, 768, Tc), (768, 3072, Tc)]  # the step's 24 problems
    jobs, base = [], []
    for M, N, Kr in shapes:
        dy = (torch.randn(Kr, M, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
        x = torch.randn(Kr, N, device="cuda", generator=g).to(torch.bfloat16)
        jobs.append((dy, x, torch.empty(M, N, device="cuda"), False))
        base.append([torch.randn(M, N, device="cuda", generator=g), torch.rand(M, N, device="cuda", generator=g) * 1e-3,
                     torch.rand(M, N, device="cuda", generator=g) * 1e-6])
    split = K._dw_tail_split(jobs)
    F = sum((M // 256) * (N // 256) for M, N, Kr in shapes if Kr == T)
    if F % K._cu_count() in range(1, K._cu_count() // 2 + 1):
        assert split is not None and sum(o.numel() for _, _, o, _ in split[0] + split[1]) == \
            sum(o.numel() for _, _, o, _ in jobs)
    arms = []
    for tail in (False, True):
        st = [[t.clone() for t in b] + [b[0].to(torch.bfloat16)] for b in base]
        step = torch.full((1,), 2, dtype=torch.int32, device="cuda")
        views = {j[2].data_ptr(): i for i, j in enumerate(jobs)}

        def adam(outs, n_wT=0, st=st, step=step):
            flat = []
            for o in outs:  # the state slice under each (possibly row-sliced) gradient view
                i = next(k for p0, k in views.items()
                         if p0 <= o.data_ptr() < p0 + jobs[k][2].numel() * 4)
                r0 = (o.data_ptr() - jobs[i][2].data_ptr()) // (4 * o.shape[1])
                flat += [t[r0:r0 + o.shape[0]] for t in st[i]]
            return flat + [step], [1e-3, 0.9, 0.999, 1e-8, 0.0, 0.0]

        old = K.DW_TAIL
        K.DW_TAIL = tail
        try:
            K.linear_dw_batch(jobs, adam=adam)
        finally:
            K.DW_TAIL = old
        torch.cuda.synchronize()
        arms.append(st)
    for a, b in zip(*arms):
        for x, y in zip(a, b):
            assert torch.equal(x, y)
