"""A training step captured as a CHAIN of HIP graphs (engine/graph.py, FD_GRAPH_SPLIT: the capture
is cut after the named blocks' forward, so a replay's first graph starts on the GPU while the host
still submits the rest) replays bit for bit like the single-graph capture and the eager steps."""
import pytest
import torch

from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.engine import (
    ArenaAdam, GraphedTrainStep, make_step_fn)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.models import (
    DDoSClassifier, DistilBertConfig)

pytestmark = pytest.mark.gpu


def _batch(B, S, seed):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(1000, 2000, (B, S), generator=g)
    lens = torch.randint(60, 85, (B,), generator=g)
    mask = (torch.arange(S)[None] < lens[:, None]).long()
    ids = ids * mask
    ids[:, 0] = 101
    labels = torch.randint(0, 2, (B,), generator=g)
    return ids.cuda(), mask.cuda(), labels.cuda(), int(lens.sum())


@pytest.mark.parametrize("split", [(0,), (0, 1)])
def test_graph_chain_matches_single_graph_and_eager(split):
    cfg = DistilBertConfig(n_layers=3)
    runs = []
    for mode in ("chain", "single", "eager"):
        m = DDoSClassifier(config=cfg, device="cuda", impl="hip", seed=12)
        m.train()
        st = GraphedTrainStep(make_step_fn(m, ArenaAdam(m, lr=1e-3)), warmup=1, enabled=mode != "eager",
                              bucket=m.packed_rows)
        st.split = split if mode == "chain" else ()
        losses = []
        for it in range(5):
            ids, mask, labels, tokens = _batch(32, 128, seed=90 + it)
            losses.append(float(st(ids, mask, labels, tokens)))
        torch.cuda.synchronize()
        assert st.failed is None
        if mode == "chain":
            assert st.graph_count == len(split) + 1
        if mode == "single":
            assert st.graph_count == 1
        runs.append((losses, m.arena.master.clone()))
    (l0, w0), (l1, w1), (l2, w2) = runs
    assert l0 == l1 and torch.equal(w0, w1)
    assert torch.equal(w0, w2) and max(abs(a - b) for a, b in zip(l0, l2)) < 1e-5
