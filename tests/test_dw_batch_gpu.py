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
    jobs, refs, brefs = [], [], []
    for i, (M, N) in enumerate(shapes):
        dy = (torch.randn(T, M, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
        x = torch.randn(T, N, device="cuda", generator=g).to(torch.bfloat16)
        acc = i % 3 == 2
        out = torch.randn(M, N, device="cuda", generator=g) if acc else torch.empty(M, N, device="cuda")
        ref = dy.float().t() @ x.float() + (out.clone() if acc else 0.0)
        # the producer-bias column sums of dy for half the problems (the qkv bias path)
        bias = None
        if i % 2 == 1:
            bias = torch.randn(M, device="cuda", generator=g) if acc else torch.full((M,), float("nan"), device="cuda")
            brefs.append((bias, dy.float().sum(0) + (bias.clone() if acc else 0.0)))
        jobs.append((dy, x, out, acc, bias))
        refs.append(ref)
    K.linear_dw_batch(jobs, cfg=cfg)
    torch.cuda.synchronize()
    for (_, _, out, _, _), ref in zip(jobs, refs):
        assert _frel(out, ref) < 1e-5, _frel(out, ref)
    for bias, bref in brefs:
        assert _frel(bias, bref) < 1e-5, _frel(bias, bref)


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


def test_batched_qkv_bias_partials_bitwise(monkeypatch):
    """The per-block qkv-bias column-sum partials computed in one launch at the end of the
    backward (model.batch_colsum, ops/kernels.py colsum_partials_batched) give bitwise the
    gradients of one partial launch per block -- including an accumulating second backward.
    (Only reachable with the dW launch's own qkv-bias sums off: K.DW_QKV_BIAS=False.)"""
    monkeypatch.setattr(K, "DW_QKV_BIAS", False)
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


def test_dw_launch_qkv_bias_matches_column_sum_pass(monkeypatch):
    """The qkv bias gradient summed by the all-layer dW launch's qkv tiles (K.DW_QKV_BIAS, the
    default) against the separate column-sum pass over dqkv: the same fp32 column sums (up to
    summation order), every other gradient bitwise, for a fresh and an accumulating backward."""
    cfg = DistilBertConfig(n_layers=3)
    grads = []
    for fused in (True, False):
        monkeypatch.setattr(K, "DW_QKV_BIAS", fused)
        m = DDoSClassifier(config=cfg, device="cuda", impl="hip", seed=31)
        m.train()
        ids, mask, labels, tokens = _batch(32, 128, seed=710)
        per = []
        for acc_step in range(2):
            if acc_step == 0:
                m.zero_grad()
            m.rng.fill_(acc_step)
            loss, _ = m.forward_loss(ids, mask, labels, tokens=tokens)
            loss.backward()
            torch.cuda.synchronize()
            per.append({k: m.arena.gview(k).clone() for k in m.arena.offsets})
        grads.append(per)
    for a, b in zip(*grads):  # after the first and after the accumulating second backward
        for k in a:
            if ".attention." in k and k.endswith("_lin.bias") and "out_lin" not in k:
                err = ((a[k] - b[k]).norm() / b[k].norm().clamp_min(1e-30)).item()
                assert err < 1e-5, (k, err)
            else:
                assert torch.equal(a[k], b[k]), k


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


def _dw_problems(layers, seed, pruned=True, T=2688):
    """The packed bs32 step's all-layer dW problems in backward order: the pruned block's lin2 / lin1
    / out_lin (K = 64 [CLS] rows) and qkv (K = T), then ``layers`` full blocks (K = T)."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    blk = [(768, 3072), (3072, 768), (768, 768), (2304, 768)]
    spec = ([(64, M, N) for M, N in blk[:3]] + [(T, *blk[3])] if pruned else []) + [(T, M, N) for _ in range(layers)
                                                                                   for M, N in blk]
    probs = []
    for Kt, M, N in spec:
        dy = (torch.randn(Kt, M, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
        x = torch.randn(Kt, N, device="cuda", generator=g).to(torch.bfloat16)
        st = [torch.randn(M * N, device="cuda", generator=g), torch.randn(M * N, device="cuda", generator=g) * 1e-3,
              torch.rand(M * N, device="cuda", generator=g) * 1e-6, torch.empty(M * N, device="cuda", dtype=torch.bfloat16)]
        probs.append((dy, x, M, N, st))
    return probs


def _run_dw(probs, mode, fused):
    old = K.ext().gemm_dwb_set_mix(mode)
    try:
        n0 = K.ext().gemm_dwb_mixed_launches()
        jobs, states = [], []
        for dy, x, M, N, st in probs:
            bias = torch.zeros(M, device="cuda") if M == 2304 else None  # the qkv bias column sums
            jobs.append((dy, x, torch.zeros(M, N, device="cuda"), False, bias))
            states.append([t.clone() for t in st])
        step = torch.full((1,), 3, dtype=torch.int32, device="cuda")

        def adam(outs):
            flat = [t for s in states[:len(outs)] for t in s]
            return flat + [step], [2e-5, 0.9, 0.999, 1e-8, 0.0, 0.0]

        K.linear_dw_batch(jobs, adam=adam if fused else None)
        torch.cuda.synchronize()
        mixed = K.ext().gemm_dwb_mixed_launches() - n0
    finally:
        K.ext().gemm_dwb_set_mix(old)
    return jobs, states, mixed


@pytest.mark.parametrize("layers,mode", [(5, 1), (2, 2)])
@pytest.mark.parametrize("fused", [False, True])
def test_mixed_tile_dw_schedule_bitwise(layers, mode, fused):
    """The all-layer dW launch's mixed schedule (gemm.hip plan_dwb_mix: long tiles in whole rounds,
    the excess as 256 x 128 half tiles, every class dealt evenly over the XCDs) against the plain
    256 x 256 schedule: every gradient, qkv-bias column sum and fused Adam state bitwise.  (5, 1): the
    bs32 step's own problem set, mixed by the default rule on a 256-CU MI355X; (2, 2): forced."""
    probs = _dw_problems(layers, seed=17 + layers)
    ja, sa, ma = _run_dw(probs, 0, fused)
    jb, sb, mb = _run_dw(probs, mode, fused)
    assert ma == 0
    if mode == 2 or torch.cuda.get_device_properties(0).multi_processor_count == 256:
        assert mb == 1, "the mixed schedule did not run"
    for (dya, xa, oa, _, ba), (_, _, ob, _, bb), s0, s1 in zip(ja, jb, sa, sb):
        if not fused:
            assert torch.equal(oa, ob)
            ref = dya.float().t() @ xa.float()
            assert _frel(oa, ref) < 1e-5
        else:
            for t0, t1 in zip(s0, s1):
                assert torch.equal(t0, t1)
        if ba is not None:
            assert torch.equal(ba, bb)
