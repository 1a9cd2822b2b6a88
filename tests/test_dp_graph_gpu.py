"""The data-parallel client's graph-captured step (parallel/dp.py GradSync over a NativeComm,
``capturable``; fed/runner.py dp_comm) executed on one GPU.

RCCL refuses two ranks on one device (profiles/r6_rccl_one_gpu_probe.txt), so the exchange here is
a single-rank communicator -- its all-reduces are identities -- but everything around it is the
real path: the per-block all-reduces issued from the backward hook on the side stream, the sparse
word-row union exchange, the join before Adam, and all of it captured into ONE HIP graph.  The
graph replays must equal the eager steps bit for bit, and the DP step must track the plain step
(a k = 1 exchange changes nothing; the DP step runs the per-block weight-gradient path and the
unfused Adam, so the comparison there is to rounding)."""
import pytest
import torch

from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.engine import (
    ArenaAdam, GraphedTrainStep, make_step_fn)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.models import (
    DDoSClassifier, DistilBertConfig)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.parallel import dp
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.parallel.rccl import (
    NativeComm)

pytestmark = pytest.mark.gpu


def _batches(n, B=16, S=128):
    g = torch.Generator().manual_seed(21)
    out = []
    for _ in range(n):
        ids = torch.randint(1000, 2000, (B, S), generator=g)
        lens = torch.randint(60, 100, (B,), generator=g)
        mask = (torch.arange(S)[None] < lens[:, None]).long()
        ids = ids * mask
        ids[:, 0] = 101
        out.append((ids.cuda(), mask.cuda(), torch.randint(0, 2, (B,), generator=g).cuda()))
    return out


def _run(kind, batches):
    m = DDoSClassifier(config=DistilBertConfig(n_layers=2), device="cuda", impl="hip", seed=12)
    m.train()
    opt = ArenaAdam(m, lr=1e-3)
    comm = sync = None
    p0 = m.arena.master.clone()
    if kind == "plain":
        fn = make_step_fn(m, opt)
        st = GraphedTrainStep(fn, warmup=1, enabled=False)
    else:
        comm = NativeComm(rank=0, world_size=1)
        sync = dp.GradSync(m, None, 1, max_rows=16 * 128, ncomm=comm)
        assert sync.capturable
        fn = dp.make_dp_step_fn(m, opt, sync)
        st = GraphedTrainStep(fn, warmup=1, enabled=(kind == "dp_graph"))
    try:
        losses = [float(st(ids, mask, labels)) for ids, mask, labels in batches]
        torch.cuda.synchronize()
        if kind == "dp_graph":
            assert st.failed is None and st.graph is not None, st.failed
        return losses, m.arena.master - p0
    finally:
        if sync is not None:
            sync.detach()
        if comm is not None:
            comm.close()


def test_dp_native_comm_step_graph_equals_eager():
    batches = _batches(4)
    l_graph, p_graph = _run("dp_graph", batches)
    l_eager, p_eager = _run("dp_eager", batches)
    l_plain, p_plain = _run("plain", batches)
    assert l_graph == l_eager and torch.equal(p_graph, p_eager)
    for a, b in zip(l_eager, l_plain):
        assert abs(a - b) < 1e-2 * abs(b), (l_eager, l_plain)
    assert ((p_eager - p_plain).norm() / p_plain.norm()).item() < 5e-2
