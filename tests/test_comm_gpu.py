"""Native RCCL communicator (csrc/comm/rccl_comm.cpp) on one GPU.

RCCL refuses two ranks on one device, so the 1-GPU box can only exercise a
single-rank communicator: it checks the binding, the run-time binding of
torch's librccl, the unique-id / init path and every collective's plumbing
(in-place results, dtypes, stream ordering).  Multi-rank FedAvg numerics are
covered by the gloo tests (tests/test_distributed_gloo.py) on the same code path.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_native_comm_single_rank_collectives():
    from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.parallel.rccl import (
        NativeComm)
    c = NativeComm(rank=0, world_size=1)
    try:
        x = torch.randn(1 << 20, device="cuda")
        ref = x.clone()
        c.all_reduce_(x, "sum")
        torch.cuda.synchronize()
        assert torch.equal(x, ref)
        c.all_reduce_(x, "avg")
        assert torch.equal(x, ref)
        y = torch.randn(1000, device="cuda").to(torch.bfloat16)
        y0 = y.clone()
        c.broadcast_(y, root=0)
        assert torch.equal(y, y0)
        g = c.all_gather(ref[:128])
        assert g.shape == (1, 128) and torch.equal(g[0], ref[:128])
        w = torch.tensor([2.5], dtype=torch.float64, device="cuda")
        c.all_reduce_(w, "max")
        assert float(w.item()) == 2.5
    finally:
        c.close()


def test_fedavg_with_native_comm_single_process():
    from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.models import (
        DDoSClassifier, DistilBertConfig)
    from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.parallel import (
        broadcast_model, fedavg_)
    from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.parallel.rccl import (
        NativeComm)
    c = NativeComm(rank=0, world_size=1)
    try:
        m = DDoSClassifier(config=DistilBertConfig(n_layers=1), device="cuda", impl="hip", seed=1)
        before = m.arena.master.clone()
        broadcast_model(m, comm=c)
        assert fedavg_(m, comm=c) == 1.0
        assert torch.equal(m.arena.master, before)
    finally:
        c.close()
