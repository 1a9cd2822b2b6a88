"""Intra-client data parallelism (parallel/dp.py) on CPU with gloo.

* 1 client x 2 replicas: after the gradient exchange each replica holds exactly the
  gradient of the client-batch mean loss (= single-process full-batch gradient).
* 2 clients x 2 replicas (world 4): the federated runner end to end -- replicas stay
  identical, FedAvg averages the two clients, only replica 0 writes client files.
"""
import json
import os
import socket

import torch
import torch.multiprocessing as mp

PKG = "detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env(rank, world, port):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})


def _batch(n=7, S=32, seed=0):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(1000, 2000, (n, S), generator=g)
    ids[:, 0] = 101
    mask = torch.ones(n, S, dtype=torch.int64)
    mask[1::2, 20:] = 0
    labels = torch.randint(0, 2, (n,), generator=g)
    return ids, mask, labels


def _model():
    from importlib import import_module
    models = import_module(f"{PKG}.models")
    cfg = models.DistilBertConfig(n_layers=1, dropout=0.0, attention_dropout=0.0)
    m = models.DDoSClassifier(config=cfg, seed=5, head_dropout=0.0, impl="torch")
    m.train()
    return m


def _grad_worker(rank, world, port, outdir):
    _env(rank, world, port)
    from importlib import import_module
    comm = import_module(f"{PKG}.parallel.comm")
    dp = import_module(f"{PKG}.parallel.dp")
    comm.init_distributed(device="cpu")
    topo = dp.make_topology(2)
    assert topo.num_clients == 1 and topo.dp_rank == rank
    m = _model()
    ids, mask, labels = _batch()
    b = {"input_ids": ids, "attention_mask": mask, "labels": labels}

    class _L:  # minimal loader: one client batch of 7 rows (unequal 4 / 3 shares)
        n, batch_size, drop_last = 7, 7, False

        def __iter__(self):
            yield b

    shard = next(iter(dp.DPShardLoader(_L(), topo.dp_rank, 2)))
    sync = dp.GradSync(m, topo.dp_group, 2)
    sync.set_loss_scale(shard["loss_scale"])
    m.zero_grad()
    loss, _ = m.forward_loss(shard["input_ids"], shard["attention_mask"], shard["labels"])
    (loss * sync.loss_scale).backward()
    sync.finish()
    torch.save(m.arena.grad.clone(), os.path.join(outdir, f"grad{rank}.pt"))
    comm.shutdown()


def test_dp_gradient_equals_full_batch(tmp_path):
    port = _free_port()
    mp.spawn(_grad_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    g0 = torch.load(tmp_path / "grad0.pt", weights_only=True)
    g1 = torch.load(tmp_path / "grad1.pt", weights_only=True)
    assert torch.equal(g0, g1)  # both replicas hold the same summed gradient
    m = _model()
    ids, mask, labels = _batch()
    m.zero_grad()
    loss, _ = m.forward_loss(ids, mask, labels)
    loss.backward()
    ref = m.arena.grad
    assert torch.allclose(g0, ref, rtol=1e-4, atol=1e-7), (g0 - ref).abs().max()


def test_shard_loader_splits_and_skips():
    from importlib import import_module
    dp = import_module(f"{PKG}.parallel.dp")
    data = import_module(f"{PKG}.data")

    class _DS:
        def __init__(self, n):
            self.input_ids = torch.arange(n * 4).view(n, 4)
            self.attention_mask = torch.ones(n, 4, dtype=torch.int64)
            self.labels = torch.arange(n)

        def __len__(self):
            return len(self.labels)

    loader = data.DeviceLoader(_DS(17), 8)  # batches of 8, 8, 1
    shards = [list(dp.DPShardLoader(loader, r, 2)) for r in range(2)]
    assert len(dp.DPShardLoader(loader, 0, 2)) == 2 == len(shards[0])  # the 1-row tail is skipped
    for b0, b1 in zip(*shards):
        assert b0["loss_scale"] + b1["loss_scale"] == 1.0
        assert set(b0["labels"].tolist()).isdisjoint(b1["labels"].tolist())


def _fed_worker(rank, world, port, outdir):
    _env(rank, world, port)
    torch.set_num_threads(max(1, 8 // world))
    from importlib import import_module
    runner = import_module(f"{PKG}.fed.runner")
    config = import_module(f"{PKG}.config")
    models = import_module(f"{PKG}.models")
    data = import_module(f"{PKG}.data")
    comm = import_module(f"{PKG}.parallel.comm")
    comm.init_distributed(device="cpu")
    cfg = config.FedConfig(out_dir=outdir, synthetic_rows=800, data_fraction=0.1, max_len=64, epochs=1,
                           batch_size=8, eval_batch_size=16, plots=False, resume=False, rounds=1,
                           verbose=False, gpus_per_client=2)
    frame = data.generate_cicids2017(cfg.synthetic_rows, seed=0)
    client = runner.FederatedClient(cfg, frame=frame, model_config=models.DistilBertConfig(n_layers=1))
    client.run()
    torch.save(client.model.arena.master.clone(), os.path.join(outdir, f"master{rank}.pt"))
    comm.shutdown()


def test_two_dp_clients_federated_run(tmp_path):
    port = _free_port()
    mp.spawn(_fed_worker, args=(4, port, str(tmp_path)), nprocs=4, join=True)
    ms = [torch.load(tmp_path / f"master{r}.pt", weights_only=True) for r in range(4)]
    for m in ms[1:]:
        assert torch.equal(ms[0], m)  # replicas identical, and FedAvg made the clients identical
    rep = json.load(open(tmp_path / "federated_report.json"))
    assert len(rep["clients"]) == 2 and rep["gpus_per_client"] == 2
    for cid in (1, 2):
        assert (tmp_path / f"client{cid}_local_metrics.csv").exists()
        assert (tmp_path / f"client{cid}_model.pth").exists()
    assert not (tmp_path / "client3_model.pth").exists()


def _kd_grad_worker(rank, world, port, outdir):
    _env(rank, world, port)
    from importlib import import_module
    comm = import_module(f"{PKG}.parallel.comm")
    dp = import_module(f"{PKG}.parallel.dp")
    comm.init_distributed(device="cpu")
    topo = dp.make_topology(2)
    m, t = _model(), _teacher()
    ids, mask, labels = _batch()
    b = {"input_ids": ids, "attention_mask": mask, "labels": labels}

    class _L:
        n, batch_size, drop_last = 7, 7, False

        def __iter__(self):
            yield b

    class _NoStep:  # keep the exchanged gradient for inspection
        overlap = False

        def zero_grad(self):
            m.zero_grad()

        def step(self):
            pass

    shard = next(iter(dp.DPShardLoader(_L(), topo.dp_rank, 2)))
    sync = dp.GradSync(m, topo.dp_group, 2)
    sync.set_loss_scale(shard["loss_scale"])
    step = dp.make_dp_step_fn(m, _NoStep(), sync, teacher=t, temperature=2.0, alpha=0.5)
    step(shard["input_ids"], shard["attention_mask"], shard["labels"])
    torch.save(m.arena.grad.clone(), os.path.join(outdir, f"kdgrad{rank}.pt"))
    comm.shutdown()


def _teacher():
    from importlib import import_module
    models = import_module(f"{PKG}.models")
    cfg = models.DistilBertConfig(n_layers=2, dropout=0.0, attention_dropout=0.0)
    t = models.BertTeacherClassifier(config=cfg, seed=11, head_dropout=0.0, impl="torch")
    t.eval()
    return t


def test_dp_distillation_gradient_equals_full_batch(tmp_path):
    """KD on a data-parallel client: the replicas' shard-weighted KD gradients sum to the
    full-batch KD gradient (same frozen teacher on every replica)."""
    from importlib import import_module
    kd_loss = import_module(f"{PKG}.models.bert").kd_loss
    port = _free_port()
    mp.spawn(_kd_grad_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    g0 = torch.load(tmp_path / "kdgrad0.pt", weights_only=True)
    g1 = torch.load(tmp_path / "kdgrad1.pt", weights_only=True)
    assert torch.equal(g0, g1)
    m, t = _model(), _teacher()
    ids, mask, labels = _batch()
    m.zero_grad()
    with torch.no_grad():
        tl = t(ids, mask)
    kd_loss(m(ids, mask), tl, labels, 2.0, 0.5).backward()
    ref = m.arena.grad
    assert torch.allclose(g0, ref, rtol=1e-4, atol=1e-7), (g0 - ref).abs().max()


def _tcp_fed_worker(rank, world, port, outdir, pr, ps):
    _env(rank, world, port)
    from importlib import import_module
    runner = import_module(f"{PKG}.fed.runner")
    config = import_module(f"{PKG}.config")
    models = import_module(f"{PKG}.models")
    data = import_module(f"{PKG}.data")
    comm = import_module(f"{PKG}.parallel.comm")
    comm.init_distributed(device="cpu")
    cfg = config.FedConfig(out_dir=outdir, synthetic_rows=800, data_fraction=0.1, max_len=64, epochs=1,
                           batch_size=8, eval_batch_size=16, plots=False, resume=False, rounds=1,
                           verbose=False, gpus_per_client=2, transport="tcp", server_host="127.0.0.1",
                           port_receive=pr, port_send=ps, timeout_s=60.0)
    frame = data.generate_cicids2017(cfg.synthetic_rows, seed=0)
    client = runner.FederatedClient(cfg, frame=frame, model_config=models.DistilBertConfig(n_layers=1))
    client.run()
    torch.save(client.model.arena.master.clone(), os.path.join(outdir, f"tcpmaster{rank}.pt"))
    comm.shutdown()


def test_two_dp_clients_over_the_reference_tcp_protocol(tmp_path):
    """2 clients x 2 replicas with the reference's star TCP exchange: one upload per client
    (replica 0), the server's mean reaches every replica of both clients."""
    import threading
    from importlib import import_module
    tp = import_module(f"{PKG}.parallel.transport")
    pr, ps = _free_port(), _free_port()
    srv = tp.FedAvgServer(2, "127.0.0.1", pr, ps, timeout=60)
    res = {}
    th = threading.Thread(target=lambda: res.setdefault("agg", srv.run_round()), daemon=True)
    th.start()
    srv.ready.wait(10)
    port = _free_port()
    mp.spawn(_tcp_fed_worker, args=(4, port, str(tmp_path), pr, ps), nprocs=4, join=True)
    th.join(60)
    ms = [torch.load(tmp_path / f"tcpmaster{r}.pt", weights_only=True) for r in range(4)]
    for m in ms[1:]:
        assert torch.equal(ms[0], m)  # every replica of both clients holds the server's mean
    assert res.get("agg") is not None and len(srv.received) == 2


def test_fused_ln_backward_off_beside_collectives():
    """while a data-parallel client's gradient all-reduces overlap the backward, the
    LayerNorm-fused backward GEMMs (whose row blocks wait for every tile to be resident) are not
    used: RCCL's kernels may hold the CUs a peer tile needs.  The rule (ops/kernels.py
    ln_fusable) and its trigger (GradSync attaching its per-block hook) are checked on CPU; the
    GPU side (no gemm_ln backward launch, same gradients) in tests/test_model_gpu.py."""
    from importlib import import_module
    K = import_module(f"{PKG}.ops.kernels")
    dp = import_module(f"{PKG}.parallel.dp")
    assert K.ln_fusable(2688, 768)
    assert not K.ln_fusable(2688, 768, concurrent_collectives=True)
    m = _model()
    assert not getattr(m, "collectives_in_backward", False)
    sync = dp.GradSync(m, None, 2)
    assert m.collectives_in_backward
    sync.detach()
    assert not m.collectives_in_backward
    dp.GradSync(m, None, 2, overlap=False)  # no per-block hook: nothing runs beside the backward
    assert not m.collectives_in_backward


def test_four_dp_clients_on_eight_ranks(tmp_path):
    """The target node's 8 ranks as 4 clients x 2 data-parallel replicas (--gpus-per-client 2): every
    replica of every client ends on the same FedAvg aggregate, and rank 0's report has 4 clients."""
    port = _free_port()
    mp.spawn(_fed_worker, args=(8, port, str(tmp_path)), nprocs=8, join=True)
    ms = [torch.load(tmp_path / f"master{r}.pt", weights_only=True) for r in range(8)]
    for m in ms[1:]:
        assert torch.equal(ms[0], m)
    rep = json.load(open(tmp_path / "federated_report.json"))
    assert len(rep["clients"]) == 4 and rep["gpus_per_client"] == 2 and rep["world_size"] == 8
    for cid in range(1, 5):
        assert (tmp_path / f"client{cid}_aggregated_metrics.csv").exists()
    assert not (tmp_path / "client5_model.pth").exists()
