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


def test_bench_refuses_too_few_gpus(monkeypatch):
    """On a box with fewer GPUs than --gpus the launcher exits non-zero instead of running (and
    reporting) fewer ranks."""
    import importlib.util
    import torch
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.delenv("FEDDDOS_BACKEND", raising=False)
    called = []
    monkeypatch.setattr(bench.subprocess, "call", lambda *a, **k: called.append(a) or 0)
    assert bench._spawn(bench._args(["--gpus", "2"])) == 2
    assert not called
