"""bench.py output contract (one JSON line with the driver's fields), on CPU with a tiny model."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_json_line():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--impl", "torch", "--layers", "1",
                          "--steps", "2", "--warmup", "1", "--batch-size", "2", "--seq-len", "64"],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["higher_is_better"] is True
    assert d["config"]["seq_len"] == 64
    # one process: the quality half still runs the reference's 2-client round (virtual clients
    # trained in turn, seeds 42 / 43), and the average is not an identity
    assert d["quality_virtual_clients"] == 2 and d["quality_clients"] == 2
    pc = d["per_client"]
    assert [c["seed"] for c in pc] == [42, 43]
    assert all(c["rel_l2_local_to_aggregate"] > 0 for c in pc)
    assert d["eval_rows"] == sum(c["test_rows"] for c in pc)


def test_bench_spawns_ranks_itself():
    """--gpus 2 without a torchrun environment: bench.py starts 2 ranks as a child
    torch.distributed.run, every rank checks WORLD_SIZE, rank 0 prints the one line with the
    FedAvg round of the quality protocol (gloo on CPU)."""
    env = dict(os.environ, FEDDDOS_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--impl", "torch",
                          "--layers", "1", "--steps", "2", "--warmup", "1", "--batch-size", "2", "--seq-len", "64"],
                         capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["fedavg_rounds"] == 1 and d["quality_clients"] == 2
    assert len(d["per_rank_ms_per_step"]) == 2 and d["backend"] == "gloo"
    assert d["eval_rows"] == 2 * d["eval_rows_per_client"]
    assert d["allreduce_bytes"] > 0 and d["fedavg_ms"] is not None


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    return bench


def _fake_kfd(tmp_path, gpu_ids):
    for i, g in enumerate(gpu_ids):
        d = tmp_path / "nodes" / str(i)
        d.mkdir(parents=True)
        (d / "gpu_id").write_text(f"{g}\n")
    return str(tmp_path / "nodes")


def test_bench_refuses_too_few_gpus(monkeypatch, tmp_path):
    """On a box with fewer GPUs than --gpus the launcher exits non-zero instead of running (and
    reporting) fewer ranks.  The GPUs are counted from the KFD sysfs topology -- never through
    torch / HIP, so the launcher parent never initialises the GPU runtime."""
    import torch
    bench = _bench_module()
    nodes = _fake_kfd(tmp_path, [0, 51234])  # one CPU node, one GPU node
    monkeypatch.setattr(bench, "KFD_NODES", nodes)
    monkeypatch.setattr(bench._visible_gpus, "__defaults__", (nodes,))
    monkeypatch.setattr(torch.cuda, "device_count", lambda: (_ for _ in ()).throw(AssertionError("GPU library")))
    monkeypatch.delenv("FEDDDOS_BACKEND", raising=False)
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    called = []
    monkeypatch.setattr(bench.subprocess, "call", lambda *a, **k: called.append(a) or 0)
    assert bench._spawn(bench._args(["--gpus", "2"])) == 2
    assert not called


def test_visible_gpu_count_from_sysfs(monkeypatch, tmp_path):
    bench = _bench_module()
    nodes = _fake_kfd(tmp_path, [0] * 2 + [1000 + i for i in range(8)])  # 2 CPU sockets, 8 GPUs
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    assert bench._visible_gpus(nodes) == 8
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2,3")
    assert bench._visible_gpus(nodes) == 4
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "5")
    assert bench._visible_gpus(nodes) == 1
    monkeypatch.setenv("CUDA_VISIBLE_DEVICES", "")
    assert bench._visible_gpus(nodes) == 0
    assert bench._visible_gpus(str(tmp_path / "missing")) == 0


def test_bench_eight_clients_gloo():
    """The 8-rank path the driver's scaling run takes, rehearsed on CPU (gloo, tiny model): eight
    per-rank times, eight clients in the FedAvg round and the quality protocol, the pooled eval
    rows = 8 x one client's, and the parent never opened a GPU."""
    env = dict(os.environ, FEDDDOS_BACKEND="gloo", OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--impl", "torch",
                          "--layers", "1", "--steps", "2", "--warmup", "1", "--batch-size", "2", "--seq-len", "64",
                          "--quality-rows", "1200"],
                         capture_output=True, text=True, timeout=900, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["quality_clients"] == 8 and d["fedavg_rounds"] == 1
    assert len(d["per_rank_ms_per_step"]) == 8 and d["backend"] == "gloo"
    assert d["eval_rows"] == 8 * d["eval_rows_per_client"] and d["eval_rows_per_client"] > 0
    assert d["config"]["parallelism"] == "fedavg8 (1 client/GPU)" and d["config"]["global_batch"] == 16
    assert d["parent_gpu_initialized"] is False


def test_cli_scaling_curve(tmp_path):
    """``cli scaling`` runs bench.py per GPU count (bench starts its own ranks on a free port: two
    curves can run at once) and writes the per-client efficiency vs 1 GPU."""
    env = dict(os.environ, FEDDDOS_BACKEND="gloo", OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    out_json = tmp_path / "scaling.json"
    out = subprocess.run([sys.executable, "-m",
                          "detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd",
                          "scaling", "--gpus", "1,2", "--steps", "2", "--warmup", "1", "--out", str(out_json),
                          "--impl", "torch", "--layers", "1", "--batch-size", "2", "--seq-len", "64",
                          "--quality-rows", "600"], capture_output=True, text=True, timeout=900, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    res = json.loads(out_json.read_text())
    assert [r["n_gpus"] for r in res] == [1, 2]
    assert res[0]["per_client_efficiency_vs_1gpu"] == 1.0
