"""HIP DistilBERT path vs the pure-torch fp32 path on identical weights and dropout masks."""
import pytest
import torch

from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.models import (
    DDoSClassifier, DistilBertConfig)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.engine import ArenaAdam

pytestmark = pytest.mark.gpu


def _batch(B, S, seed=0):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(1000, 2000, (B, S), generator=g)
    lens = torch.randint(S // 2, S + 1, (B,), generator=g)
    mask = (torch.arange(S)[None] < lens[:, None]).long()
    ids = ids * mask
    ids[:, 0] = 101
    labels = torch.randint(0, 2, (B,), generator=g)
    return ids.cuda(), mask.cuda(), labels.cuda()


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-8)).item()


@pytest.mark.parametrize("train", [False, True])
def test_hip_matches_torch_forward_backward(train):
    cfg = DistilBertConfig(n_layers=2)
    hip = DDoSClassifier(config=cfg, device="cuda", impl="hip", seed=3)
    ref = DDoSClassifier(config=cfg, device="cuda", impl="torch", seed=3)
    ids, mask, labels = _batch(4, 128)
    hip.train(train)
    ref.train(train)
    # same dropout counter on both paths
    hip.rng.zero_()
    ref.torch_counter = 0
    hip.zero_grad()
    ref.zero_grad()
    lh, zh = hip.forward_loss(ids, mask, labels)
    lr_, zr = ref.forward_loss(ids, mask, labels)
    assert rel(zh, zr) < 5e-2
    lh.backward()
    lr_.backward()
    gh, gr = hip.arena.grad, ref.arena.grad
    assert rel(gh, gr) < 8e-2  # first backward: untouched word rows are still zero
    for name in ["classifier.weight", "distilbert.transformer.layer.1.ffn.lin2.weight",
                 "distilbert.transformer.layer.0.attention.q_lin.weight",
                 "distilbert.embeddings.word_embeddings.weight", "distilbert.embeddings.position_embeddings.weight"]:
        assert rel(hip.dense_grad(name), ref.arena.gview(name)) < 1e-1, name


def test_state_dict_roundtrip_and_shadow_sync():
    m = DDoSClassifier(config=DistilBertConfig(n_layers=1), device="cuda", impl="hip", seed=1)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m2 = DDoSClassifier(config=DistilBertConfig(n_layers=1), device="cuda", impl="hip", seed=2)
    m2.load_state_dict(sd)
    ids, mask, _ = _batch(2, 64)
    m.eval(); m2.eval()
    with torch.no_grad():
        assert torch.equal(m(ids, mask), m2(ids, mask))


def test_training_reduces_loss_and_graph_capture():
    from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.engine import (
        GraphedTrainStep, make_step_fn)
    m = DDoSClassifier(config=DistilBertConfig(n_layers=2), device="cuda", impl="hip", seed=0)
    opt = ArenaAdam(m, lr=1e-4)
    step = GraphedTrainStep(make_step_fn(m, opt), warmup=2)
    ids, mask, labels = _batch(8, 128, seed=5)
    m.train()
    losses = [float(step(ids, mask, labels)) for _ in range(12)]
    assert step.graph is not None, step.failed
    assert losses[-1] < losses[0]


def test_full_size_step_is_finite():
    """bs32 x seq128 full model, several graphed steps: loss stays finite (workspace sizing at T = 4096)."""
    from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.engine import (
        GraphedTrainStep, make_step_fn)
    m = DDoSClassifier(device="cuda", impl="hip", seed=0)
    opt = ArenaAdam(m, lr=2e-5)
    step = GraphedTrainStep(make_step_fn(m, opt), warmup=1)
    ids, mask, labels = _batch(32, 128, seed=7)
    m.train()
    losses = [float(step(ids, mask, labels)) for _ in range(4)]
    assert all(l == l and abs(l) < 100 for l in losses), losses
    assert torch.isfinite(m.arena.master).all()


def test_teacher_hip_matches_torch_and_kd_graph_step():
    from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.models import (
        BertTeacherClassifier, bert_base_config)
    from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.engine import (
        GraphedTrainStep, make_kd_step_fn)
    th = BertTeacherClassifier(config=bert_base_config(n_layers=2), device="cuda", impl="hip", seed=4)
    tt = BertTeacherClassifier(config=bert_base_config(n_layers=2), device="cuda", impl="torch", seed=4)
    ids, mask, labels = _batch(4, 128, seed=3)
    th.eval(); tt.eval()
    with torch.no_grad():
        assert rel(th(ids, mask), tt(ids, mask)) < 5e-2
    student = DDoSClassifier(config=DistilBertConfig(n_layers=2), device="cuda", impl="hip", seed=0)
    opt = ArenaAdam(student, lr=1e-4)
    step = GraphedTrainStep(make_kd_step_fn(student, th, opt, 2.0, 0.5), warmup=2)
    student.train()
    losses = [float(step(ids, mask, labels)) for _ in range(8)]
    assert step.graph is not None, step.failed
    assert all(l == l for l in losses) and losses[-1] < losses[0]


def test_plain_forward_logits_are_differentiable():
    """model(ids, mask) + an external criterion (the reference's API) backpropagates on the HIP path."""
    m = DDoSClassifier(config=DistilBertConfig(n_layers=1), device="cuda", impl="hip", seed=0)
    r = DDoSClassifier(config=DistilBertConfig(n_layers=1), device="cuda", impl="torch", seed=0)
    ids, mask, labels = _batch(4, 64, seed=1)
    m.eval(); r.eval()
    crit = torch.nn.CrossEntropyLoss()
    m.zero_grad(); r.zero_grad()
    crit(m(ids, mask), labels).backward()
    crit(r(ids, mask), labels).backward()
    assert rel(m.dense_grad("classifier.weight"), r.arena.gview("classifier.weight")) < 5e-2


@pytest.mark.parametrize("graph", [False, True])
def test_overlapped_adam_matches_single_pass(graph):
    """Per-block Adam on a side stream during backward == one Adam pass after backward (bitwise)."""
    from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.engine import (
        GraphedTrainStep, make_step_fn)
    cfg = DistilBertConfig(n_layers=3)
    models, steps = [], []
    for overlap in (True, False):
        m = DDoSClassifier(config=cfg, device="cuda", impl="hip", seed=5)
        m.fuse_colsum = False  # (a per-block hook disables the deferred sums it needs)
        m.batch_dw = False     # (... and the all-layer weight-gradient launch)
        m.train()
        opt = ArenaAdam(m, lr=1e-3, overlap=overlap, fuse_dw=False)
        assert (m.layer_grads_hook is not None) == overlap
        models.append(m)
        steps.append(GraphedTrainStep(make_step_fn(m, opt), warmup=1, enabled=graph))
    for it in range(4):
        ids, mask, labels = _batch(8, 128, seed=it)
        for st in steps:
            st(ids, mask, labels)
    torch.cuda.synchronize()
    assert torch.equal(models[0].arena.master, models[1].arena.master)
    assert torch.equal(models[0].arena.shadow, models[1].arena.shadow)
    if graph:
        assert all(st.graph is not None for st in steps)


def test_training_is_bitwise_deterministic():
    """identical seeds + batches -> bitwise-identical weights and losses
    (no float atomics on any reduction path: split-K slabs, column partials and the
    embedding-gradient rank sort all reduce in a fixed order)."""
    from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.engine import (
        GraphedTrainStep, make_step_fn)
    runs = []
    for _ in range(2):
        m = DDoSClassifier(config=DistilBertConfig(n_layers=2), device="cuda", impl="hip", seed=9)
        m.train()
        st = GraphedTrainStep(make_step_fn(m, ArenaAdam(m, lr=1e-3)), warmup=1)
        losses = []
        for it in range(4):
            ids, mask, labels = _batch(16, 128, seed=100 + it)
            losses.append(st(ids, mask, labels).clone())
        torch.cuda.synchronize()
        runs.append((torch.stack(losses), m.arena.master.clone(), m.arena.grad.clone()))
    assert torch.equal(runs[0][0], runs[1][0])
    assert torch.equal(runs[0][1], runs[1][1])
    assert torch.equal(runs[0][2], runs[1][2])


def test_deferred_colsum_matches_immediate():
    """All bias / LN-affine column sums finalised in one batched launch at the end of the
    backward == each finalised right after its producer (bitwise; same fixed-order sum)."""
    cfg = DistilBertConfig(n_layers=2)
    grads = []
    for defer in (True, False):
        m = DDoSClassifier(config=cfg, device="cuda", impl="hip", seed=12)
        m.defer_colsum = defer
        m.fuse_colsum = False  # (the fused lin1-bias sum has its own order: test below)
        m.train()
        ids, mask, labels = _batch(16, 128, seed=300)
        for acc_step in range(2):  # second backward accumulates (deferred jobs carry the flag)
            if acc_step == 0:
                m.zero_grad()
            loss, _ = m.forward_loss(ids, mask, labels)
            loss.backward()
        torch.cuda.synchronize()
        grads.append(m.arena.grad.clone())
    assert torch.equal(grads[0], grads[1])


@pytest.mark.parametrize("tokens", [False, True])
def test_deferred_dw_reduce_matches_immediate(tokens):
    """Split-K weight-gradient slabs of the whole backward reduced in one batched launch at
    the end == each reduced right after its GEMM (bitwise; same z order), including an
    accumulating second backward and the packed-token path (K = packed rows)."""
    from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import (
        kernels as K)
    cfg = DistilBertConfig(n_layers=2)
    grads = []
    for defer in (True, False):
        m = DDoSClassifier(config=cfg, device="cuda", impl="hip", seed=12)
        m.batch_dw = False  # the per-layer grouped launches are the path under test
        m.defer_dw_reduce = defer
        m.train()
        ids, mask, labels = _batch(16, 128, seed=301)
        tok = int(mask.sum()) if tokens else None
        for acc_step in range(2):
            if acc_step == 0:
                m.zero_grad()
            loss, _ = m.forward_loss(ids, mask, labels, tokens=tok)
            loss.backward()
        torch.cuda.synchronize()
        grads.append(m.arena.grad.clone())
    # the out_lin + qkv pair does split at these shapes, so the deferred path was exercised
    assert K.ext().gemm_dw2_splits(768, 768, 2304, 768, 16 * 128) > 1
    assert torch.equal(grads[0], grads[1])


def test_fused_lin1_bias_colsum_matches_separate_pass():
    """lin1's bias gradient summed in the GELU' dX GEMM epilogue == the separate column-sum
    pass (same bf16 values, different fp32 summation order); every other gradient bitwise."""
    cfg = DistilBertConfig(n_layers=2)
    grads = []
    for fuse in (True, False):
        m = DDoSClassifier(config=cfg, device="cuda", impl="hip", seed=14)
        m.fuse_colsum = fuse
        m.train()
        ids, mask, labels = _batch(16, 128, seed=302)
        m.zero_grad()
        loss, _ = m.forward_loss(ids, mask, labels, tokens=int(mask.sum()))
        loss.backward()
        torch.cuda.synchronize()
        grads.append(m.arena.grad.clone())
    sel = torch.zeros_like(grads[0], dtype=torch.bool)
    for i in range(cfg.n_layers):
        off, shape = m.arena.offsets[f"distilbert.transformer.layer.{i}.ffn.lin1.bias"]
        sel[off:off + shape[0]] = True
        a, b = grads[0][off:off + shape[0]], grads[1][off:off + shape[0]]
        assert rel(a, b) < 1e-5, rel(a, b)
    assert torch.equal(grads[0][~sel], grads[1][~sel])


@pytest.mark.parametrize("graph", [False, True])
def test_remat_gelu_matches_saved_activation(graph):
    """The backward re-creating the FFN activation gelu(u) in the GELU' dX epilogue
    (RunCtx.remat_gelu, FD_REMAT_GELU=1) gives bitwise the gradients and weights of keeping it."""
    from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.engine import (
        GraphedTrainStep, make_step_fn)
    cfg = DistilBertConfig(n_layers=2)
    models, steps = [], []
    for remat in (True, False):
        m = DDoSClassifier(config=cfg, device="cuda", impl="hip", seed=13)
        m.remat_gelu = remat
        m.train()
        models.append(m)
        steps.append(GraphedTrainStep(make_step_fn(m, ArenaAdam(m, lr=1e-3)), warmup=1, enabled=graph))
    for it in range(3):
        ids, mask, labels = _batch(16, 128, seed=300 + it)
        for st in steps:
            st(ids, mask, labels)
    torch.cuda.synchronize()
    assert torch.equal(models[0].arena.grad, models[1].arena.grad)
    assert torch.equal(models[0].arena.master, models[1].arena.master)


def test_fused_kd_head_matches_torch_kd_loss():
    """The distillation loss fused into the head kernel == eager kd_loss on the fp32 path."""
    hip = DDoSClassifier(config=DistilBertConfig(n_layers=2), device="cuda", impl="hip", seed=21)
    ref = DDoSClassifier(config=DistilBertConfig(n_layers=2), device="cuda", impl="torch", seed=21)
    ids, mask, labels = _batch(8, 128, seed=9)
    t_logits = torch.randn(8, 2, device="cuda") * 2
    for m in (hip, ref):
        m.train()
        m.zero_grad()
    hip.rng.zero_()
    ref.torch_counter = 0
    lh, zh = hip.forward_loss(ids, mask, labels, kd=(t_logits, 2.0, 0.3))
    lr_, zr = ref.forward_loss(ids, mask, labels, kd=(t_logits, 2.0, 0.3))
    lh.backward()
    lr_.backward()
    assert abs(lh.item() - lr_.item()) < 2e-2 * max(1.0, abs(lr_.item()))
    for name in ("classifier.weight", "distilbert.transformer.layer.1.ffn.lin2.weight"):
        a, b = hip.dense_grad(name), ref.arena.gview(name)
        assert ((a - b).norm() / b.norm()).item() < 3e-2, name


def test_teacher_token_type_grad_hip_matches_torch():
    from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.models import (
        BertTeacherClassifier, bert_base_config)
    th = BertTeacherClassifier(config=bert_base_config(n_layers=2), device="cuda", impl="hip", seed=4)
    tt = BertTeacherClassifier(config=bert_base_config(n_layers=2), device="cuda", impl="torch", seed=4)
    ids, mask, labels = _batch(8, 128, seed=3)
    for m in (th, tt):
        m.train()
        m.zero_grad()
    th.rng.zero_()
    tt.torch_counter = 0
    th.forward_loss(ids, mask, labels)[0].backward()
    tt.forward_loss(ids, mask, labels)[0].backward()
    name = "distilbert.embeddings.token_type_embeddings.weight"
    a, b = th.arena.gview(name), tt.arena.gview(name)
    assert b[0].norm() > 0 and a[1].abs().sum() == 0
    assert ((a[0] - b[0]).norm() / b[0].norm()).item() < 3e-2


def test_no_fused_ln_backward_beside_collectives(monkeypatch):
    """With collectives overlapping the backward (parallel/dp.py GradSync sets
    ``collectives_in_backward``) the model runs no LayerNorm-fused dX GEMM (their
    row-block rendezvous needs every tile resident, RCCL kernels could hold the CUs), and the
    gradients equal the fused path's to bf16 accuracy."""
    from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as kn
    ids, mask, labels = _batch(B=16, S=128)  # 2,048 padded rows: a fusable (one-round) grid
    grads = []
    for beside in (False, True):
        model = DDoSClassifier(config=DistilBertConfig(n_layers=2), device="cuda", impl="hip", seed=3)
        model.train()
        model.collectives_in_backward = beside
        calls = []
        real = kn.linear_dx_ln_bwd

        def spy(*a, **k):
            calls.append(a[0].shape[0])
            return real(*a, **k)

        monkeypatch.setattr(kn, "linear_dx_ln_bwd", spy)
        model.zero_grad()
        loss, _ = model.forward_loss(ids, mask, labels)
        loss.backward()
        torch.cuda.synchronize()
        monkeypatch.setattr(kn, "linear_dx_ln_bwd", real)
        full = [m for m in calls if m > 64]  # (the pruned block's M = 64 split-K call has no rendezvous)
        assert (len(full) == 0) == beside, calls
        grads.append(model.arena.grad.clone())
    g0, g1 = grads
    assert ((g0 - g1).norm() / g0.norm()).item() < 2e-2


def test_eval_graphs_survive_interleaved_training():
    """Round 4 regression: the bs16 eval forward's HIP graphs keep valid buffers while bs32 training
    steps run between their replays (a per-shape buffer set of the pruned last block used to be
    replaced -- freed -- by the other shape; a second virtual client's eval then faulted).  The
    replayed logits equal an eager forward's bit for bit."""
    from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.engine import (
        make_step_fn)
    from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.engine.infer import (
        GraphedForward)
    model = DDoSClassifier(config=DistilBertConfig(n_layers=2), device="cuda", impl="hip", seed=3)
    opt = ArenaAdam(model, lr=1e-4)
    fn = make_step_fn(model, opt)
    ids32, mask32, lab32 = _batch(32, 128)
    ids16, mask16, _ = _batch(16, 128, seed=5)
    tok32, tok16 = int(mask32.sum()), int(mask16.sum())
    fwd = GraphedForward(model)
    for _ in range(3):
        model.train()
        fn(ids32, mask32, lab32, tok32)
        out = fwd(ids16, mask16, tok16).clone()  # capture on the first pass, replays after
        with torch.no_grad():
            model.eval()
            ref = model(ids16, mask16, tokens=tok16)
        torch.cuda.synchronize()
        assert torch.equal(out, ref)


