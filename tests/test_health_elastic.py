"""Failure detection (parallel/health.py) and elastic recovery, on CPU with gloo.

* A rank that dies is named by the survivors' health-checked barrier within a
  few seconds (the reference would block 300 s in accept, server.py:119).
* ``cli launch --max-restarts 1`` with a client killed at round 2: the group is
  restarted, every client resumes from the last completed round and the job
  finishes both rounds.
"""
import json
import os
import socket
import subprocess
import sys
import time

import torch.multiprocessing as mp

PKG = "detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir, dead=1):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    from importlib import import_module
    comm = import_module(f"{PKG}.parallel.comm")
    health = import_module(f"{PKG}.parallel.health")
    comm.init_distributed(device="cpu")
    import torch
    torch.set_num_threads(1)
    mon = health.start(interval=0.2, stale_s=2.0, timeout_s=60.0)
    mon.barrier("warm")  # everyone alive: passes
    if rank == dead:
        mon.stop()
        time.sleep(30)  # hangs without beating (a wedged process looks the same as a dead one)
        os._exit(0)
    t0 = time.monotonic()
    try:
        mon.barrier("never")
        res = "no failure detected"
    except health.PeerFailure as e:
        res = f"dead={e.dead} after {time.monotonic() - t0:.1f}s"
    with open(os.path.join(outdir, f"result{rank}.txt" if world > 2 else "result.txt"), "w") as f:
        f.write(res)
    if rank == 0 and world > 2:
        # rank 0 hosts the TCPStore: stay up until every survivor has recorded its verdict
        t_end = time.monotonic() + 60
        while time.monotonic() < t_end and not all(
                os.path.exists(os.path.join(outdir, f"result{r}.txt")) for r in range(world) if r != dead):
            time.sleep(0.1)
    os._exit(0)


def test_dead_peer_detected_fast(tmp_path):
    port = _free_port()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in ps:
        p.start()
    ps[0].join(90)
    for p in ps:
        if p.is_alive():
            p.kill()
    res = (tmp_path / "result.txt").read_text()
    assert res.startswith("dead=[1]"), res
    assert float(res.split("after ")[1][:-1]) < 15


def test_dead_peer_detected_fast_eight_ranks(tmp_path):
    """N = 8 (the target node): rank 5 wedges; EVERY survivor names it within seconds."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_worker, args=(r, 8, port, str(tmp_path), 5)) for r in range(8)]
    for p in ps:
        p.start()
    for r, p in enumerate(ps):
        if r != 5:
            p.join(120)
    for p in ps:
        if p.is_alive():
            p.kill()
    for r in range(8):
        if r == 5:
            continue
        res = (tmp_path / f"result{r}.txt").read_text()
        assert res.startswith("dead=[5]"), (r, res)
        assert float(res.split("after ")[1][:-1]) < 20


def test_elastic_restart_resumes_round(tmp_path):
    env = dict(os.environ, FEDDDOS_KILL_CLIENT="1", FEDDDOS_KILL_ROUND="1", PYTHONPATH=ROOT,
               CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", PKG, "launch", "--nproc", "2", "--port", str(_free_port()), "--max-restarts", "1",
           "--out-dir", str(tmp_path), "--synthetic-rows", "600", "--max-len", "64", "--epochs", "1",
           "--batch-size", "8", "--eval-batch-size", "32", "--rounds", "2", "--plots", "false", "--layers", "1",
           "--heartbeat-s", "0.2", "--heartbeat-stale-s", "3"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=540)
    log = out.stdout + out.stderr
    assert out.returncode == 0, log[-3000:]
    assert (tmp_path / ".killed_client1_round1_r0").exists()  # the fault did fire once
    assert "elastic restart #1" in log
    for cid in (1, 2):
        st = json.load(open(tmp_path / f"client{cid}_fed_state.json"))
        assert st["completed_rounds"] == 2
        assert [h["round"] for h in st["history"]] == [1, 2]


def test_elastic_restart_after_fedavg_first_round(tmp_path):
    """Client 2 dies in round 1 AFTER the FedAvg all-reduce, before it records the round
    (ranks could then resume at different rounds, or from a client's LOCAL model).
    The restarted group must agree on one resume round -- the round tag of the aggregate -- and
    finish with every client holding the same final aggregate."""
    import torch
    env = dict(os.environ, FEDDDOS_KILL_CLIENT="1", FEDDDOS_KILL_ROUND="0", FEDDDOS_KILL_AT="post_fedavg",
               PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", PKG, "launch", "--nproc", "2", "--port", str(_free_port()), "--max-restarts", "1",
           "--out-dir", str(tmp_path), "--synthetic-rows", "600", "--max-len", "64", "--epochs", "1",
           "--batch-size", "8", "--eval-batch-size", "32", "--rounds", "2", "--plots", "false", "--layers", "1",
           "--heartbeat-s", "0.2", "--heartbeat-stale-s", "3"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=540)
    log = out.stdout + out.stderr
    assert out.returncode == 0, log[-3000:]
    assert (tmp_path / ".killed_client1_round0_r0").exists()
    assert "elastic restart #1" in log
    assert json.load(open(tmp_path / "ddos_distilbert_model.json"))["round"] == 2
    for cid in (1, 2):
        st = json.load(open(tmp_path / f"client{cid}_fed_state.json"))
        assert st["completed_rounds"] == 2
        rounds = [h["round"] for h in st["history"]]
        assert rounds[-1] == 2 and rounds == sorted(set(rounds))
    g = torch.load(tmp_path / "ddos_distilbert_model.pth", weights_only=True)
    for cid in (1, 2):
        c = torch.load(tmp_path / f"client{cid}_model.pth", weights_only=True)
        assert all(torch.equal(g[k], c[k]) for k in g)


def test_elastic_restart_eight_clients(tmp_path):
    """N = 8: client 6 is killed in round 2; the restarted 8-process group resumes from the
    round-1 aggregate and all eight clients finish both rounds on the same final aggregate."""
    import torch
    env = dict(os.environ, FEDDDOS_KILL_CLIENT="5", FEDDDOS_KILL_ROUND="1", PYTHONPATH=ROOT,
               CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", PKG, "launch", "--nproc", "8", "--port", str(_free_port()), "--max-restarts", "1",
           "--out-dir", str(tmp_path), "--synthetic-rows", "600", "--max-len", "64", "--epochs", "1",
           "--batch-size", "8", "--eval-batch-size", "32", "--rounds", "2", "--plots", "false", "--layers", "1",
           "--heartbeat-s", "0.2", "--heartbeat-stale-s", "5"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    log = out.stdout + out.stderr
    assert out.returncode == 0, log[-3000:]
    assert (tmp_path / ".killed_client5_round1_r0").exists()
    assert "elastic restart #1" in log
    g = torch.load(tmp_path / "ddos_distilbert_model.pth", weights_only=True)
    for cid in range(1, 9):
        st = json.load(open(tmp_path / f"client{cid}_fed_state.json"))
        assert st["completed_rounds"] == 2, cid
        c = torch.load(tmp_path / f"client{cid}_model.pth", weights_only=True)
        assert all(torch.equal(g[k], c[k]) for k in g), cid


def _tiny_client(tmp_path):
    from importlib import import_module
    config = import_module(f"{PKG}.config")
    runner = import_module(f"{PKG}.fed.runner")
    models = import_module(f"{PKG}.models")
    cfg = config.FedConfig(out_dir=str(tmp_path), synthetic_rows=400, data_fraction=0.25, max_len=32, epochs=1,
                           batch_size=8, eval_batch_size=32, plots=False, impl="torch", use_graph=False,
                           heartbeat_s=0.0, verbose=False)
    return runner.FederatedClient(cfg, model_config=models.DistilBertConfig(n_layers=1)), models


def test_resume_legacy_untagged_out_dir(tmp_path):
    """an out_dir written before the round tag existed (aggregate on disk, sidecar
    completed_rounds > 0, no ddos_distilbert_model.json) must resume at the sidecar's round from
    the aggregate -- not silently restart at round 1 and overwrite it."""
    import torch
    from importlib import import_module
    ck = import_module(f"{PKG}.utils.checkpoint")
    client, models = _tiny_client(tmp_path)
    donor = models.DDoSClassifier(config=models.DistilBertConfig(n_layers=1), impl="torch", seed=123)
    ck.save_model(donor, ck.global_ckpt_path(str(tmp_path)))
    ck.save_fed_state(str(tmp_path), 1, {"completed_rounds": 1, "history": [{"round": 1}]})
    assert not os.path.exists(ck.global_tag_path(str(tmp_path)))
    client.setup()
    assert client.start_round == 1
    assert [h["round"] for h in client.history] == [1]
    got, want = client.model.state_dict(), donor.state_dict()
    assert all(torch.equal(got[k].cpu(), want[k].cpu()) for k in want)


def test_resume_untagged_without_sidecar_starts_fresh(tmp_path):
    """An aggregate with neither a tag nor a sidecar round: start at round 1 (logged)."""
    from importlib import import_module
    ck = import_module(f"{PKG}.utils.checkpoint")
    client, models = _tiny_client(tmp_path)
    donor = models.DDoSClassifier(config=models.DistilBertConfig(n_layers=1), impl="torch", seed=123)
    ck.save_model(donor, ck.global_ckpt_path(str(tmp_path)))
    client.setup()
    assert client.start_round == 0
