"""Multi-GPU RCCL correctness: 2 ranks, one GPU each, backend "nccl" (= RCCL over xGMI).

Self-skips below 2 visible GPUs (the development box has one; the driver's 8-GPU node runs
it).  What the first multi-GPU run must prove before any scaling number means anything:

* ``NativeComm`` (csrc/comm/rccl_comm.cpp): all-reduce sum / avg, broadcast and all-gather
  against exactly known values;
* ``fedavg_`` over RCCL -- with torch.distributed's communicator AND with NativeComm -- is the
  bit-exact mean of two different arenas (server.py:67-79 semantics: unweighted mean), and the
  bf16 compute shadow is refreshed from it;
* a data-parallel client (2 GPUs, ``GradSync``: per-block async all-reduces from the backward
  hook + the compacted sparse word-row exchange) gives the full-batch gradient;
* the data-parallel step over a group ``NativeComm`` replays from a HIP graph bitwise equal to
  the eager step (the collectives are side-stream ordered and captured with the step);
* a peer that dies inside FedAvg: the survivor's ``NativeComm`` collective does not hang -- its
  bounded wait (ncclCommGetAsyncError polling) aborts the communicator (ncclCommAbort) and raises
  ``PeerFailure`` within the timeout (reference: 300 s socket timeouts, server.py:10).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

PKG = "detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd"
pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs >= 2 GPUs (RCCL, one rank per GPU)")]


def _batch(dev, n=16, S=64):
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(1000, 1400, (n, S), generator=g)
    ids[:, 0] = 101
    mask = torch.ones(n, S, dtype=torch.int64)
    mask[1::2, 40:] = 0
    ids[mask == 0] = 0
    labels = torch.randint(0, 2, (n,), generator=g)
    return ids.to(dev), mask.to(dev), labels.to(dev)


def _real_batch(dev, n=64, S=128):
    """bs32 x seq128 per rank at the real data's sentence lengths (~76-96 tokens + padding)."""
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(1000, 29000, (n, S), generator=g)
    ids[:, 0] = 101
    lens = torch.randint(76, 97, (n,), generator=g)
    mask = (torch.arange(S)[None, :] < lens[:, None]).to(torch.int64)
    ids[mask == 0] = 0
    labels = torch.randint(0, 2, (n,), generator=g)
    return ids.to(dev), mask.to(dev), labels.to(dev)


def _model(dev, real=False):
    from importlib import import_module
    models = import_module(f"{PKG}.models")
    if real:  # the flagship: 6 layers, hidden / attention / head dropout on
        m = models.DDoSClassifier(config=models.DistilBertConfig(), seed=7, device=dev, impl="hip")
    else:
        cfg = models.DistilBertConfig(n_layers=2, dropout=0.0, attention_dropout=0.0)
        m = models.DDoSClassifier(config=cfg, seed=7, head_dropout=0.0, device=dev, impl="hip")
    m.train()
    return m


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    os.environ.pop("FEDDDOS_BACKEND", None)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    from importlib import import_module
    comm = import_module(f"{PKG}.parallel.comm")
    di = comm.init_distributed(timeout_s=120)
    assert di.backend == "nccl" and di.device.index == rank
    return comm, di


def _comm_worker(rank, world, port, outdir):
    comm, di = _init(rank, world, port)
    from importlib import import_module
    NativeComm = import_module(f"{PKG}.parallel.rccl").NativeComm
    c = NativeComm()
    res = {}
    x = torch.arange(1 << 20, dtype=torch.float32, device="cuda") * (rank + 1)
    base = torch.arange(1 << 20, dtype=torch.float32, device="cuda")
    c.all_reduce_(x, "sum")
    res["sum"] = torch.equal(x, base * sum(r + 1 for r in range(world)))
    y = torch.full((4096,), float(2 * rank + 1), device="cuda")
    c.all_reduce_(y, "avg")
    res["avg"] = torch.equal(y, torch.full_like(y, float(world)))
    z = torch.full((1000,), float(rank + 7), device="cuda").to(torch.bfloat16)
    c.broadcast_(z, root=1)
    res["bcast"] = torch.equal(z, torch.full_like(z, 8.0))
    g = c.all_gather(torch.full((16,), float(rank), device="cuda"))
    res["gather"] = all(torch.equal(g[r], torch.full((16,), float(r), device="cuda")) for r in range(world))
    torch.cuda.synchronize()
    c.close()
    torch.save(res, os.path.join(outdir, f"comm{rank}.pt"))
    comm.shutdown()


def _fedavg_worker(rank, world, port, outdir, which):
    comm, di = _init(rank, world, port)
    from importlib import import_module
    models = import_module(f"{PKG}.models")
    fedavg = import_module(f"{PKG}.parallel.fedavg")
    nc = import_module(f"{PKG}.parallel.rccl").NativeComm() if which == "rccl" else None
    m = models.DDoSClassifier(config=models.DistilBertConfig(n_layers=1), device="cuda", impl="hip", seed=40 + rank)
    torch.save(m.arena.master.cpu(), os.path.join(outdir, f"before{rank}.pt"))
    total = fedavg.fedavg_(m, comm=nc)
    torch.cuda.synchronize()
    torch.save({"after": m.arena.master.cpu(), "shadow": m.arena.shadow.cpu(), "total": total},
               os.path.join(outdir, f"after{rank}.pt"))
    if nc is not None:
        nc.close()
    comm.shutdown()


def _dp_worker(rank, world, port, outdir):
    comm, di = _init(rank, world, port)
    from importlib import import_module
    dp = import_module(f"{PKG}.parallel.dp")
    topo = dp.make_topology(2)
    m = _model(di.device)
    ids, mask, labels = _batch(di.device)
    sl = slice(8 * rank, 8 * rank + 8)
    sync = dp.GradSync(m, topo.dp_group, 2, max_rows=16 * 64)
    sync.set_loss_scale(0.5)
    m.zero_grad()
    loss, _ = m.forward_loss(ids[sl], mask[sl], labels[sl])
    (loss * sync.loss_scale).backward()
    hooked = len(sync.done)
    sync.finish()
    torch.cuda.synchronize()
    torch.save({"grad": m.arena.grad.cpu(), "now": m.emb_now.cpu(), "hooked": hooked},
               os.path.join(outdir, f"dp{rank}.pt"))
    comm.shutdown()


def _dp_graph_worker(rank, world, port, outdir, real=False):
    """The same data-parallel training steps eager and replayed from a HIP graph: GradSync over a
    NativeComm of the client's group (side-stream collectives, no host sync) is capturable.
    ``real``: the flagship 6-layer model at bs32 x seq128 per rank with dropout on -- the grids
    the driver's scaling bench runs (252-tile LayerNorm-fused forwards beside RCCL's kernels)."""
    comm, di = _init(rank, world, port)
    from importlib import import_module
    dp = import_module(f"{PKG}.parallel.dp")
    rccl = import_module(f"{PKG}.parallel.rccl")
    engine = import_module(f"{PKG}.engine")
    K = import_module(f"{PKG}.ops.kernels")
    topo = dp.make_topology(2)
    nc = rccl.NativeComm(group=topo.dp_group)
    n = 32 if real else 8
    ids, mask, labels = (_real_batch if real else _batch)(di.device)
    sl = slice(n * rank, n * rank + n)
    out = {}
    for graphed in (False, True):
        m = _model(di.device, real)
        opt = engine.ArenaAdam(m, lr=1e-3)
        sync = dp.GradSync(m, topo.dp_group, 2, max_rows=2 * n * ids.shape[1], ncomm=nc)
        assert sync.capturable
        sync.set_loss_scale(0.5)
        step = engine.GraphedTrainStep(dp.make_dp_step_fn(m, opt, sync), warmup=2, enabled=graphed)
        losses = [step(ids[sl], mask[sl], labels[sl]).clone() for _ in range(5)]
        torch.cuda.synchronize()
        out["graph" if graphed else "eager"] = {"master": m.arena.master.cpu(), "loss": torch.stack(losses).cpu(),
                                                "captured": step.graph is not None, "failed": str(step.failed),
                                                "ln_error": K.ln_error_flag(di.device)}
        sync.detach()
        del step, opt, m
    nc.close()
    torch.save(out, os.path.join(outdir, f"dpg{rank}.pt"))
    comm.shutdown()


def _abort_worker(rank, world, port, outdir):
    import time
    comm, di = _init(rank, world, port)
    from importlib import import_module
    rccl = import_module(f"{PKG}.parallel.rccl")
    health = import_module(f"{PKG}.parallel.health")
    c = rccl.NativeComm(timeout_s=20.0)
    x = torch.ones(1 << 24, dtype=torch.float32, device="cuda")
    c.all_reduce_(x, "sum")  # healthy round first: both ranks present
    ok = torch.equal(x, torch.full_like(x, 2.0))
    comm.barrier()
    if rank == 1:
        os._exit(0)  # dies "mid-FedAvg": the next collective has one participant only
    t0 = time.monotonic()
    try:
        c.all_reduce_(x, "sum")
        res = "no failure detected"
    except health.PeerFailure as e:
        res = f"raised after {time.monotonic() - t0:.1f}s: {e}"
    with open(os.path.join(outdir, "abort.txt"), "w") as f:
        f.write(f"{ok}|{res}|{c.handle}")
    os._exit(0)  # (the process group's peer is gone: no collective shutdown)


def _spawn(fn, *args, world=2, timeout=180):
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=fn, args=(r, world, port) + args) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_native_comm_two_ranks(tmp_path):
    _spawn(_comm_worker, str(tmp_path))
    for r in range(2):
        res = torch.load(tmp_path / f"comm{r}.pt", weights_only=True)
        assert all(res.values()), res


@pytest.mark.parametrize("which", ["torch", "rccl"])
def test_fedavg_bit_exact_mean_over_rccl(tmp_path, which):
    _spawn(_fedavg_worker, str(tmp_path), which)
    b0 = torch.load(tmp_path / "before0.pt", weights_only=True)
    b1 = torch.load(tmp_path / "before1.pt", weights_only=True)
    assert not torch.equal(b0, b1)
    mean = (b0 + b1) * 0.5  # a + b then x0.5 is exact-rounded the same way as RCCL's sum then 1/N
    for r in range(2):
        a = torch.load(tmp_path / f"after{r}.pt", weights_only=True)
        assert a["total"] == 2.0
        assert torch.equal(a["after"], mean)
        assert torch.equal(a["shadow"], mean.to(torch.bfloat16))


def test_dp_gradsync_matches_full_batch_over_rccl(tmp_path):
    _spawn(_dp_worker, str(tmp_path))
    r0 = torch.load(tmp_path / "dp0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "dp1.pt", weights_only=True)
    assert r0["hooked"] == 2 and torch.equal(r0["now"], r1["now"])
    dev = torch.device("cuda")
    m = _model(dev)
    ids, mask, labels = _batch(dev)
    m.zero_grad()
    loss, _ = m.forward_loss(ids, mask, labels)
    loss.backward()
    torch.cuda.synchronize()
    ref = m.arena.grad.cpu()
    woff, V, D = m.word_embedding_span()
    rows = m.emb_now.cpu().bool()
    for r in (r0, r1):
        g = r["grad"]
        gw, rw = g[woff:woff + V * D].view(V, D), ref[woff:woff + V * D].view(V, D)
        assert torch.allclose(gw[rows], rw[rows], rtol=2e-2, atol=2e-5)
        g2, ref2 = g.clone(), ref.clone()
        g2[woff:woff + V * D] = 0
        ref2[woff:woff + V * D] = 0
        assert ((g2 - ref2).norm() / ref2.norm()).item() < 2e-2
    # replicas hold the same summed gradient (word rows outside the batch are never written)
    assert torch.equal(r0["grad"][woff + V * D:], r1["grad"][woff + V * D:])
    assert torch.equal(r0["grad"][:woff], r1["grad"][:woff])


@pytest.mark.parametrize("real", [False, True], ids=["toy", "6layer_bs32_seq128"])
def test_dp_step_graphed_equals_eager_over_native_comm(tmp_path, real):
    _spawn(_dp_graph_worker, str(tmp_path), real, timeout=300)
    r = [torch.load(tmp_path / f"dpg{i}.pt", weights_only=True) for i in range(2)]
    for x in r:
        assert x["graph"]["captured"] and x["graph"]["failed"] == "None", x["graph"]["failed"]
        assert not x["eager"]["captured"]
        # no LayerNorm-fused rendezvous timed out beside the gradient all-reduces
        assert x["graph"]["ln_error"] == 0 and x["eager"]["ln_error"] == 0
        # same kernels in the same order on the same inputs: the replayed step is the eager step
        assert torch.equal(x["graph"]["master"], x["eager"]["master"])
        assert torch.equal(x["graph"]["loss"], x["eager"]["loss"])
    # the replicas stay identical (summed gradients, identical Adam)
    assert torch.equal(r[0]["graph"]["master"], r[1]["graph"]["master"])


def test_dead_peer_in_fedavg_aborts_instead_of_hanging(tmp_path):
    _spawn(_abort_worker, str(tmp_path), timeout=150)
    ok, res, handle = (tmp_path / "abort.txt").read_text().split("|")
    assert ok == "True"
    assert res.startswith("raised after"), res
    assert float(res.split("after ")[1].split("s")[0]) < 60, res
    assert handle == "0"  # aborted
