"""Data-parallel client on the HIP path (one GPU, two replicas, gloo between them).

RCCL refuses two ranks on one device, so the box's single MI355X hosts both
replicas and gloo carries the exchange; the code under test is the HIP-path
specific part of parallel/dp.py: per-block all-reduces launched from the
backward hook and the compacted sparse word-embedding row exchange.  The summed
gradient must match one process running the whole client batch.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

PKG = "detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batch(dev, n=16, S=64):
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(1000, 1400, (n, S), generator=g)
    ids[:, 0] = 101
    mask = torch.ones(n, S, dtype=torch.int64)
    mask[1::2, 40:] = 0
    ids[mask == 0] = 0
    labels = torch.randint(0, 2, (n,), generator=g)
    return ids.to(dev), mask.to(dev), labels.to(dev)


def _model(dev):
    from importlib import import_module
    models = import_module(f"{PKG}.models")
    cfg = models.DistilBertConfig(n_layers=2, dropout=0.0, attention_dropout=0.0)
    m = models.DDoSClassifier(config=cfg, seed=7, head_dropout=0.0, device=dev, impl="hip")
    m.train()
    return m


def _worker(rank, world, port, outdir):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": "0",
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "FEDDDOS_BACKEND": "gloo"})
    from importlib import import_module
    comm = import_module(f"{PKG}.parallel.comm")
    dp = import_module(f"{PKG}.parallel.dp")
    di = comm.init_distributed()
    topo = dp.make_topology(2)
    m = _model(di.device)
    ids, mask, labels = _batch(di.device)
    sl = slice(8 * rank, 8 * rank + 8)
    sync = dp.GradSync(m, topo.dp_group, 2, max_rows=16 * 64)
    sync.set_loss_scale(0.5)
    m.zero_grad()
    loss, _ = m.forward_loss(ids[sl], mask[sl], labels[sl])
    (loss * sync.loss_scale).backward()
    n_hooked = len(sync.done)
    sync.finish()
    torch.cuda.synchronize()
    K = import_module(f"{PKG}.ops.kernels")
    assert K._SHARED_DEVICE  # two ranks on one GPU: no kernel may assume it owns every CU
    torch.save({"grad": m.arena.grad.cpu(), "now": m.emb_now.cpu(), "hooked": n_hooked},
               os.path.join(outdir, f"dp{rank}.pt"))
    comm.shutdown()


def test_dp_hip_gradient_matches_full_batch(tmp_path):
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(150)
        assert p.exitcode == 0, f"replica exit code {p.exitcode}"
    r0 = torch.load(tmp_path / "dp0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "dp1.pt", weights_only=True)
    assert r0["hooked"] == 2  # both blocks were exchanged from the backward hook
    assert torch.equal(r0["now"], r1["now"])
    dev = torch.device("cuda")
    # the replicas shared this GPU, so they ran the separate LayerNorm kernels (ops/kernels.py
    # set_shared_device: a fused-LN grid may not own every CU there); the reference takes the same
    # kernels, so the comparison is of the exchange, not of two LayerNorm roundings
    from importlib import import_module
    K = import_module(f"{PKG}.ops.kernels")
    K.set_shared_device(True)
    try:
        m = _model(dev)
        ids, mask, labels = _batch(dev)
        m.zero_grad()
        loss, _ = m.forward_loss(ids, mask, labels)
        loss.backward()
        torch.cuda.synchronize()
    finally:
        K.set_shared_device(False)
    now = m.emb_now.cpu()
    assert torch.equal(now, r0["now"])  # union of replica rows == rows of the full batch
    woff, V, D = m.word_embedding_span()
    ref = m.arena.grad.cpu().clone()
    rows = now.bool()
    for r in (r0, r1):
        g = r["grad"]
        gw, rw = g[woff:woff + V * D].view(V, D), ref[woff:woff + V * D].view(V, D)
        assert torch.allclose(gw[rows], rw[rows], rtol=2e-2, atol=2e-5), (gw[rows] - rw[rows]).abs().max()
        g2, r2 = g.clone(), ref.clone()
        g2[woff:woff + V * D] = 0
        r2[woff:woff + V * D] = 0
        err = (g2 - r2).norm() / r2.norm()
        assert err < 2e-2, float(err)
    assert torch.equal(r0["grad"][woff + V * D:], r1["grad"][woff + V * D:])
