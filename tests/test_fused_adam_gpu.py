"""Adam fused into the weight-gradient GEMM epilogues == gradient, then Adam kernel.

The fused epilogue (csrc/kernels/gemm.hip ``adam_epi4``) runs the Adam kernel's
arithmetic on the finished fp32 gradient tile (a fused launch never splits K).  So a
fused training step reproduces the unfused one bit for bit when the unfused one does
not split K either.
"""
import pytest
import torch

from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.engine import (
    ArenaAdam, GraphedTrainStep, make_step_fn)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.models import (
    DDoSClassifier, DistilBertConfig)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _batch(B, S, seed=0):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(1000, 2000, (B, S), generator=g)
    lens = torch.randint(S // 3, S + 1, (B,), generator=g)
    mask = (torch.arange(S)[None] < lens[:, None]).long()
    ids = ids * mask
    ids[:, 0] = 101
    labels = torch.randint(0, 2, (B,), generator=g)
    return ids.cuda(), mask.cuda(), labels.cuda(), int(lens.sum())


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-8)).item()


@pytest.fixture
def nosplit():
    """Weight-gradient GEMMs unsplit in both arms (a fused launch never splits K; a split
    unfused one would sum in another fp32 order)."""
    K.ext().gemm_set_cfg(2, -1, 1)
    yield
    K.ext().gemm_set_cfg(2, -1, -1)


@pytest.mark.parametrize("graph", [False, True])
def test_fused_adam_training_matches_unfused(graph, nosplit):
    cfg = DistilBertConfig(n_layers=2)
    models, opts, steps = [], [], []
    for fuse in (True, False):
        m = DDoSClassifier(config=cfg, device=DEV, impl="hip", seed=13)
        m.train()
        opt = ArenaAdam(m, lr=1e-3, fuse_dw=fuse)
        assert opt.can_fuse() == fuse
        models.append(m)
        opts.append(opt)
        steps.append(GraphedTrainStep(make_step_fn(m, opt), warmup=1, enabled=graph, bucket=m.packed_rows))
    losses = [[], []]
    for it in range(5):
        ids, mask, labels, tokens = _batch(16, 128, seed=300 + it)
        for i, st in enumerate(steps):
            losses[i].append(float(st(ids, mask, labels, tokens)))
    torch.cuda.synchronize()
    assert models[0].fused_opt is None  # the scope ended with the step
    a, b = models[0].arena, models[1].arena
    # every fused span must be skipped by step() and updated exactly once by a GEMM
    assert opts[0]._done == [] and int(opts[0].step_t) == 5  # (host_step counts eager calls only)
    assert torch.equal(opts[0].step_t, opts[1].step_t)
    assert losses[0] == losses[1]
    assert torch.equal(a.master, b.master), rel(a.master, b.master)
    assert torch.equal(opts[0].m, opts[1].m) and torch.equal(opts[0].v, opts[1].v)
    assert torch.equal(a.shadow, b.shadow)
    if graph:
        assert all(st.graph is not None and st.failed is None for st in steps)


def test_fused_adam_touches_only_encoder_matrices():
    """The fused spans are exactly the 4 weight matrices of every block; the bias / LN /
    embedding / head parameters are left to the run-table Adam launch."""
    cfg = DistilBertConfig(n_layers=2)
    m = DDoSClassifier(config=cfg, device=DEV, impl="hip", seed=3)
    m.train()
    opt = ArenaAdam(m, lr=1e-3, fuse_dw=True)
    seen = []
    orig = opt.fused_args

    def spy(grads):
        out = orig(grads)
        seen.extend(opt._done[-len(grads):])
        return out
    opt.fused_args = spy
    ids, mask, labels, tokens = _batch(8, 128, seed=1)
    make_step_fn(m, opt)(ids, mask, labels, tokens)
    torch.cuda.synchronize()
    want = set()
    for i in range(cfg.n_layers):
        pre = f"distilbert.transformer.layer.{i}."
        q, _ = m.arena.offsets[pre + "attention.q_lin.weight"]
        want.add((q, 3 * 768 * 768))
        for nm in ("attention.out_lin.weight", "ffn.lin1.weight", "ffn.lin2.weight"):
            off, shape = m.arena.offsets[pre + nm]
            want.add((off, shape[0] * shape[1]))
    assert set(seen) == want and len(seen) == len(want)


@pytest.mark.parametrize("shapes,T", [(((768, 3072), (3072, 768)), 2688)])  # one K split either way
def test_dw_fused_adam_matches_gradient_then_adam(shapes, T):
    _check_fused_dw(shapes, T)


def _check_fused_dw(shapes, T):
    """One grouped dW launch with Adam in the epilogue == dW into fp32 gradients + the Adam kernel."""
    (M0, N0), (M1, N1) = shapes
    g = torch.Generator(device=DEV).manual_seed(5)

    def bf(*s):
        return (torch.randn(*s, device=DEV, generator=g) * 0.5).to(torch.bfloat16)
    dy0, x0, dy1, x1 = bf(T, M0), bf(T, N0), bf(T, M1), bf(T, N1)
    n0, n1 = M0 * N0, M1 * N1
    state = []
    for _ in range(2):
        p = torch.randn(n0 + n1, device=DEV, generator=g)
        state.append([p, torch.rand(n0 + n1, device=DEV, generator=g) * 1e-3,
                      torch.rand(n0 + n1, device=DEV, generator=g) * 1e-6, p.to(torch.bfloat16)])
    state[1] = [t.clone() for t in state[0]]
    step = torch.tensor([3], dtype=torch.int32, device=DEV)
    hp = [1e-3, 0.9, 0.999, 1e-8, 0.0, 0.0]
    # reference: gradients, then the flat Adam kernel
    grad = torch.empty(n0 + n1, device=DEV)
    K.linear_dw2(dy0, x0, grad[:n0].view(M0, N0), dy1, x1, grad[n0:].view(M1, N1))
    p, m_, v_, sh = state[1]
    K.adam(p, grad, m_, v_, sh, step, *hp[:5], False)
    # fused
    p, m_, v_, sh = state[0]
    st = [p[:n0], m_[:n0], v_[:n0], sh[:n0], p[n0:], m_[n0:], v_[n0:], sh[n0:], step]
    junk = torch.full((n0 + n1,), 7.0, device=DEV)
    K.linear_dw2(dy0, x0, junk[:n0].view(M0, N0), dy1, x1, junk[n0:].view(M1, N1), adam=(st, hp))
    torch.cuda.synchronize()
    assert (junk == 7.0).all()  # the gradient itself is never stored
    for a, b in zip(state[0], state[1]):
        assert torch.equal(a, b), rel(a, b)


@pytest.mark.parametrize("shapes,T", [(((768, 768), (2304, 768)), 2688)])
def test_dw_fused_adam_splitk_shape(shapes, T, nosplit):
    """A shape the unfused launch would split K on: the fused launch runs it unsplit."""
    _check_fused_dw(shapes, T)


def test_splitk_graph_replays_and_accumulates():
    """Split-K weight gradient (fp32 slabs + the reduce launch): repeated launches and graph
    replays give bitwise the same result; accumulate adds onto the existing gradient."""
    T, M, N = 4096, 768, 768  # 72 tiles -> split K
    g = torch.Generator(device=DEV).manual_seed(9)
    dy = (torch.randn(T, M, device=DEV, generator=g)).to(torch.bfloat16)
    x = (torch.randn(T, N, device=DEV, generator=g)).to(torch.bfloat16)
    ref = dy.float().t() @ x.float()
    out = torch.empty(M, N, device=DEV)
    K.linear_dw(dy, x, out)
    first = out.clone()
    assert rel(out, ref) < 2e-3
    K.linear_dw(dy, x, out, accumulate=True)
    assert rel(out, 2 * ref) < 2e-3
    gr = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        K.linear_dw(dy, x, out)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(gr):
        K.linear_dw(dy, x, out)
    for _ in range(3):
        out.fill_(-1.0)
        gr.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, first)


def test_adam_run_table_matches_per_run_launches():
    n = 1 << 16
    g = torch.Generator(device=DEV).manual_seed(2)
    base = [torch.randn(n, device=DEV, generator=g) for _ in range(2)] + \
        [torch.rand(n, device=DEV, generator=g) * 1e-4, torch.rand(n, device=DEV, generator=g) * 1e-6]
    runs = [(0, 4096), (8192, 64), (20000, 4), (40000, 25536)]
    a = [t.clone() for t in base]
    b = [t.clone() for t in base]
    sha, shb = a[0].to(torch.bfloat16), b[0].to(torch.bfloat16)
    step = torch.tensor([2], dtype=torch.int32, device=DEV)
    K.adam(a[0], a[1], a[2], a[3], sha, step, 1e-3, 0.9, 0.999, 1e-8, 0.0, False,
           runs=K.adam_runs(runs, DEV))
    for off, ln in runs:
        sl = slice(off, off + ln)
        K.adam(b[0][sl], b[1][sl], b[2][sl], b[3][sl], shb[sl], step, 1e-3, 0.9, 0.999, 1e-8, 0.0, False)
    torch.cuda.synchronize()
    for x, y in zip(a + [sha], b + [shb]):
        assert torch.equal(x, y)
    untouched = torch.ones(n, dtype=torch.bool, device=DEV)
    for off, ln in runs:
        untouched[off:off + ln] = False
    assert torch.equal(a[0][untouched], base[0][untouched])


def test_adam_rows_matches_flagged_dense_adam():
    """The word-embedding update by row flags (adam_rows: one wave per 64 row flags) is bitwise
    the dense launch that skips unflagged rows: rows with state but no gradient this step take
    the g = 0 update, rows without state are left untouched."""
    rows, rl = 1000, 768
    n = rows * rl
    g = torch.Generator(device=DEV).manual_seed(4)
    base = [torch.randn(n, device=DEV, generator=g), torch.randn(n, device=DEV, generator=g),
            torch.rand(n, device=DEV, generator=g) * 1e-3, torch.rand(n, device=DEV, generator=g) * 1e-6]
    ever = (torch.rand(rows, device=DEV, generator=g) < 0.2).to(torch.uint8)
    now = ((torch.rand(rows, device=DEV, generator=g) < 0.5).to(torch.uint8) * ever).contiguous()
    a = [t.clone() for t in base]
    b = [t.clone() for t in base]
    sha, shb = a[0].to(torch.bfloat16), b[0].to(torch.bfloat16)
    step = torch.tensor([3], dtype=torch.int32, device=DEV)
    K.adam_rows(a[0], a[1], a[2], a[3], sha, step, 1e-3, 0.9, 0.999, 1e-8, ever, now, rl)
    K.adam(b[0], b[1], b[2], b[3], shb, step, 1e-3, 0.9, 0.999, 1e-8, 0.0, False, ever, now, 0, rows, rl)
    torch.cuda.synchronize()
    for x, y in zip(a + [sha], b + [shb]):
        assert torch.equal(x, y)
    untouched = ever.repeat_interleave(rl) == 0
    assert torch.equal(a[0][untouched], base[0][untouched])


def test_graph_replay_after_load_state_dict_uses_loaded_weights():
    """A captured training step holds no shadow sync of its own: ``GraphedTrainStep`` brings the
    bf16 shadow up to date before each replay (``DDoSClassifier.prepare_replay``).  A graphed model
    and an eager twin take the same steps, both load the same modified checkpoint, and the next
    step (a replay on one, eager on the other) must give the same loss and the same weights --
    a replay that read the pre-load shadow would not."""
    arms = []
    for graph in (True, False):
        m = DDoSClassifier(config=DistilBertConfig(n_layers=2), device=DEV, impl="hip", seed=3)
        m.train()
        opt = ArenaAdam(m, lr=1e-3)
        arms.append((m, GraphedTrainStep(make_step_fn(m, opt), warmup=1, enabled=graph, bucket=m.packed_rows)))
    ids, mask, labels, tokens = _batch(32, 128, seed=1)
    for _ in range(3):  # graphed arm: eager, capture, replay
        losses = [float(st(ids, mask, labels, tokens)) for _, st in arms]
        assert losses[0] == losses[1]
    assert arms[0][1].graph is not None
    sd = {k: v.clone() for k, v in arms[0][0].state_dict().items()}
    sd["distilbert.transformer.layer.1.ffn.lin2.weight"].mul_(-3.0)
    sd["distilbert.transformer.layer.0.attention.q_lin.weight"].add_(0.05)
    for m, _ in arms:
        m.load_state_dict(sd)
    losses = [float(st(ids, mask, labels, tokens)) for _, st in arms]
    torch.cuda.synchronize()
    assert losses[0] == losses[1]
    a, b = arms[0][0].arena, arms[1][0].arena
    assert torch.equal(a.master, b.master) and torch.equal(a.shadow, b.shadow)
    assert torch.equal(a.shadow, a.master.to(torch.bfloat16))


@pytest.mark.parametrize("graph", [False, True])
def test_rest_of_step_in_dw_launch_bitwise(graph, monkeypatch):
    """The rest of the optimizer step (biases, LayerNorms, embeddings, head, flagged word rows)
    run by extra blocks of the all-layer dW launch and the qkv bias by its summing tiles
    (ops/kernels.py ADAM_IN_DW) == the separate adam_rows + run-table launches after it: masters,
    moments and the bf16 shadow bitwise equal after graph-replayed steps."""
    states = []
    for in_dw in (True, False):
        monkeypatch.setattr(K, "ADAM_IN_DW", in_dw)
        m = DDoSClassifier(config=DistilBertConfig(n_layers=2), device=DEV, impl="hip", seed=17)
        m.train()
        opt = ArenaAdam(m, lr=1e-3)
        calls = []
        real = K.adam
        monkeypatch.setattr(K, "adam", lambda *a, **k: (calls.append(1), real(*a, **k))[1])
        step = GraphedTrainStep(make_step_fn(m, opt), warmup=1, enabled=graph, bucket=m.packed_rows)
        for it in range(4):
            ids, mask, labels, tokens = _batch(32, 128, seed=40 + it)
            step(ids, mask, labels, tokens)
        torch.cuda.synchronize()
        monkeypatch.setattr(K, "adam", real)
        assert (len(calls) == 0) == in_dw  # (eager launches only: replays bypass Python)
        states.append((m.arena.master.clone(), opt.m.clone(), opt.v.clone(), m.arena.shadow.clone()))
    for x, y in zip(*states):
        assert torch.equal(x, y)
