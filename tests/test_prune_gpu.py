"""Last-block [CLS] pruning (RunCtx.prune_idx, ops/functional.py LayerFn._forward_pruned): the
last block runs out-proj / FFN / LayerNorms on the [CLS] rows only.  Exact by construction (no
other row of its output reaches the loss), so the logits and loss match the unpruned model and
every gradient matches up to fp32 summation order; a few graph-replayed Adam steps stay together."""
import pytest
import torch

from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.engine import (
    ArenaAdam, GraphedTrainStep, make_step_fn)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.models import (
    DDoSClassifier, DistilBertConfig)

pytestmark = pytest.mark.gpu


def _batch(B, S, seed=0):
    # CICIDS2017-like lengths (<= 84 tokens): the full model's LayerNorm-fused GEMMs stay fused
    # (<= 2,688 rows), so both arms run the same LayerNorm kernels and the forward is bitwise equal
    gen = torch.Generator().manual_seed(seed)
    ids = torch.randint(1000, 2000, (B, S), generator=gen)
    lens = torch.randint(60, 85, (B,), generator=gen)
    mask = (torch.arange(S)[None] < lens[:, None]).long()
    ids = ids * mask
    ids[:, 0] = 101
    labels = torch.randint(0, 2, (B,), generator=gen)
    return ids.cuda(), mask.cuda(), labels.cuda(), int(lens.sum())


def _frel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("packed,B", [(True, 32), (False, 16), (True, 20)])
def test_pruned_last_block_matches_full(packed, B):
    cfg = DistilBertConfig(n_layers=3)
    outs = []
    for prune in (True, False):
        m = DDoSClassifier(config=cfg, device="cuda", impl="hip", seed=31)
        m.prune_last = prune
        m.train()
        ids, mask, labels, tokens = _batch(B, 128, seed=800)
        m.zero_grad()
        m.rng.fill_(5)
        loss, logits = m.forward_loss(ids, mask, labels, tokens=tokens if packed else None)
        loss.backward()
        torch.cuda.synchronize()
        outs.append((loss.detach().clone(), logits.detach().clone(), m.arena.grad.clone(),
                     {k: m.dense_grad(k).clone() for k in m.state_dict()}))
    (l0, z0, g0, d0), (l1, z1, g1, d1) = outs
    assert torch.equal(z0, z1), (z0 - z1).abs().max()
    assert l0.item() == l1.item()
    assert _frel(g0, g1) < 1e-5
    for k in d1:
        if d1[k].norm() > 0:
            assert _frel(d0[k], d1[k]) < 1e-4, k


def test_pruned_eval_logits_match():
    cfg = DistilBertConfig(n_layers=2)
    res = []
    for prune in (True, False):
        m = DDoSClassifier(config=cfg, device="cuda", impl="hip", seed=33)
        m.prune_last = prune
        m.eval()
        ids, mask, _, tokens = _batch(32, 128, seed=801)
        with torch.no_grad():
            res.append(m(ids, mask, tokens=tokens).clone())
    assert torch.equal(res[0], res[1])


def test_pruned_graph_training_tracks_full():
    cfg = DistilBertConfig(n_layers=2)
    models, steps = [], []
    for prune in (True, False):
        m = DDoSClassifier(config=cfg, device="cuda", impl="hip", seed=35)
        m.prune_last = prune
        m.train()
        opt = ArenaAdam(m, lr=1e-4)
        models.append(m)
        steps.append(GraphedTrainStep(make_step_fn(m, opt), warmup=1, enabled=True, bucket=m.packed_rows))
    losses = [[], []]
    for it in range(6):
        ids, mask, labels, tokens = _batch(32, 128, seed=900 + it)
        for j, st in enumerate(steps):
            losses[j].append(float(st(ids, mask, labels, tokens)))
    torch.cuda.synchronize()
    assert all(st.graph is not None and st.failed is None for st in steps)
    for a, b in zip(*losses):
        assert abs(a - b) < 1e-3 * max(1.0, abs(b))
    assert _frel(models[0].arena.master, models[1].arena.master) < 1e-6
