"""The one-process R-round virtual-client protocol (fed/runner.py run_virtual_clients, used by
``bench.py --virtual-clients N --rounds R`` on one GPU) against the real N-process collective run
(``run_federated`` over gloo): for N = 2, R = 2 on a 1-layer model they must agree BIT FOR BIT --
the same per-client data, loader permutations, dropout counters, fresh Adam per round and the same
FedAvg arithmetic (an exact two-term sum, then the 1/N scale).

Reference: a FedAvg round is a re-run of the client scripts from the server's aggregate
(client1.py:375-380 resume + fresh Adam; server.py:67-79 unweighted mean)."""
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


def _cfg(config, outdir, rounds):
    return config.FedConfig(out_dir=outdir, synthetic_rows=1500, data_fraction=0.1, max_len=64, epochs=1,
                            batch_size=8, eval_batch_size=16, plots=False, resume=False, rounds=rounds,
                            verbose=False, heartbeat_s=0.0)


def _worker(rank, world, port, outdir, rounds):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    from importlib import import_module
    runner = import_module(f"{PKG}.fed.runner")
    config = import_module(f"{PKG}.config")
    models = import_module(f"{PKG}.models")
    data = import_module(f"{PKG}.data")
    comm = import_module(f"{PKG}.parallel.comm")
    comm.init_distributed(device="cpu")
    torch.set_num_threads(1)  # (CPU GEMM blocking depends on the thread count: same count both sides)
    cfg = _cfg(config, outdir, rounds)
    frame = data.generate_cicids2017(cfg.synthetic_rows, seed=0)
    runner.run_federated(cfg, frame=frame, model_config=models.DistilBertConfig(n_layers=1))
    comm.shutdown()


def test_virtual_rounds_equal_gloo_run_bitwise(tmp_path):
    world, rounds = 2, 2
    real = tmp_path / "real"
    real.mkdir()
    mp.spawn(_worker, args=(world, _free_port(), str(real), rounds), nprocs=world, join=True)

    from importlib import import_module
    runner = import_module(f"{PKG}.fed.runner")
    config = import_module(f"{PKG}.config")
    models = import_module(f"{PKG}.models")
    data = import_module(f"{PKG}.data")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        os.environ.pop(k, None)
    cfg = _cfg(config, str(tmp_path / "virtual"), rounds)
    cfg.save_checkpoints = False
    frame = data.generate_cicids2017(cfg.synthetic_rows, seed=0)
    nthreads = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        client = runner.FederatedClient(cfg, frame=frame, model_config=models.DistilBertConfig(n_layers=1)).setup()
        res = runner.run_virtual_clients(client, world, rounds=rounds)
    finally:
        torch.set_num_threads(nthreads)
    assert len(res["rounds"]) == rounds

    # the final aggregate, bit for bit
    g = torch.load(real / "ddos_distilbert_model.pth", weights_only=True)
    sd = client.model.state_dict()
    assert set(g) == set(sd)
    for key in g:
        assert torch.equal(g[key], sd[key].to(g[key].dtype)), key
    # every round's per-client local and aggregated test metrics
    for cid in range(1, world + 1):
        st = json.load(open(real / f"client{cid}_fed_state.json"))
        assert st["completed_rounds"] == rounds
        for r in range(rounds):
            want = st["history"][r]
            got = res["rounds"][r]["clients"][cid - 1]
            for key in ("local_test", "aggregated_test"):
                assert got[key]["confusion_matrix"] == want[key]["confusion_matrix"], (cid, r, key)
                assert got[key]["loss"] == want[key]["loss"], (cid, r, key)
            assert got["train"]["epoch_losses"] == want["train"]["epoch_losses"], (cid, r)
    # round 2 starts from round 1's aggregate: the local models of round 2 moved away from it
    assert res["rounds"][1]["clients"][0]["rel_l2_local_to_aggregate"] > 0


def test_virtual_rounds_bookkeeping(tmp_path):
    """3 clients x 2 rounds: per-round pooled confusion = the sum of the clients' matrices, the
    clients' dropout counters are kept per client across rounds, and round 1 alone reproduces a
    1-round run."""
    from importlib import import_module
    runner = import_module(f"{PKG}.fed.runner")
    config = import_module(f"{PKG}.config")
    models = import_module(f"{PKG}.models")
    data = import_module(f"{PKG}.data")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        os.environ.pop(k, None)
    cfg = _cfg(config, str(tmp_path), 2)
    cfg.save_checkpoints = False
    frame = data.generate_cicids2017(cfg.synthetic_rows, seed=0)

    def run(rounds):
        nthreads = torch.get_num_threads()
        torch.set_num_threads(1)  # (bitwise run-to-run comparison below)
        try:
            client = runner.FederatedClient(cfg, frame=frame,
                                            model_config=models.DistilBertConfig(n_layers=1)).setup()
            msgs = []
            return runner.run_virtual_clients(client, 3, rounds=rounds, progress=msgs.append), msgs, client
        finally:
            torch.set_num_threads(nthreads)

    two, msgs, client = run(2)
    assert len(msgs) == 2 * 3 + 2
    for h in two["rounds"]:
        cm = [[sum(c["aggregated_test"]["confusion_matrix"][i][j] for c in h["clients"]) for j in range(2)]
              for i in range(2)]
        assert cm == h["aggregated_confusion"]
        assert sum(map(sum, cm)) == sum(c["test_rows"] for c in h["clients"])
    assert two["clients"] is two["rounds"][-1]["clients"]
    one, _, _ = run(1)
    for a, b in zip(one["rounds"][0]["clients"], two["rounds"][0]["clients"]):
        assert a["aggregated_test"] == b["aggregated_test"] and a["local_test"] == b["local_test"]
    # every client ran 1 epoch per round: the last client's counter advanced by its own steps only
    steps = two["rounds"][0]["clients"][-1]["train"]["steps"]
    assert client.model.torch_counter == 2 * steps


def test_virtual_cli_writes_per_round_artifacts(tmp_path):
    """``python -m <pkg> virtual --clients 3 --rounds 2``: the one-process N x R protocol from the
    command line -- per-client, per-round CSVs in the reference schema, the tagged final aggregate
    and the JSON report."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", PKG, "virtual", "--clients", "3", "--rounds", "2", "--out-dir", str(tmp_path),
           "--synthetic-rows", "600", "--max-len", "64", "--epochs", "1", "--batch-size", "8",
           "--eval-batch-size", "32", "--plots", "false", "--layers", "1", "--verbose", "false",
           "--warm-start-epochs", "1"]
    out = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, (out.stdout + out.stderr)[-3000:]
    for k in (1, 2, 3):
        for name in ("local_metrics.csv", "aggregated_metrics.csv", "local_metrics_round2.csv",
                     "aggregated_metrics_round2.csv"):
            assert (tmp_path / f"client{k}_{name}").exists(), (k, name)
    rep = json.load(open(tmp_path / "virtual_report.json"))
    assert rep["clients"] == 3 and [r["round"] for r in rep["rounds"]] == [1, 2]
    assert rep["warm_start"]["epochs"] == 1 and "accuracy" in rep["warm_start"]["public_test"]
    assert all(len(r["clients"]) == 3 for r in rep["rounds"])
    assert json.load(open(tmp_path / "ddos_distilbert_model.json"))["round"] == 2
    assert (tmp_path / "ddos_distilbert_model.pth").exists()


def test_warm_start_is_a_shared_pretrained_point(tmp_path):
    """fed/runner.py warm_start: trains the shared init on a separate public synthetic file (no client
    samples it), then resets the dropout counters -- every virtual client starts from those weights
    exactly as from a loaded checkpoint."""
    from importlib import import_module
    runner = import_module(f"{PKG}.fed.runner")
    config = import_module(f"{PKG}.config")
    models = import_module(f"{PKG}.models")
    data = import_module(f"{PKG}.data")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        os.environ.pop(k, None)
    cfg = _cfg(config, str(tmp_path), 1)
    cfg.save_checkpoints = False
    frame = data.generate_cicids2017(cfg.synthetic_rows, seed=0)
    client = runner.FederatedClient(cfg, frame=frame, model_config=models.DistilBertConfig(n_layers=1)).setup()
    before = client.model.arena.master.clone()
    rec = runner.warm_start(client, epochs=1, rows=600)
    after = client.model.arena.master.clone()
    assert not torch.equal(before, after)
    assert rec["train"]["steps"] > 0 and 0.0 <= rec["public_test"]["accuracy"] <= 100.0
    assert client.model.torch_counter == 0 and int(client.model.rng.item()) == 0
    res = runner.run_virtual_clients(client, 2, rounds=1)
    # both clients started from the warm weights: their local models moved away from them
    assert res["rounds"][0]["clients"][0]["rel_l2_local_to_aggregate"] > 0
