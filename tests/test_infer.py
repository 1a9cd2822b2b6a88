"""Serving path: ``predict`` CLI on CPU, and the HIP-graph forward == eager forward on GPU."""
import json
import os
import subprocess
import sys

import pytest
import torch

PKG = "detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_predict_cli_writes_predictions(tmp_path):
    from importlib import import_module
    models = import_module(f"{PKG}.models")
    ck = import_module(f"{PKG}.utils.checkpoint")
    m = models.DDoSClassifier(seed=3)  # full-size, random weights: checks the checkpoint format round trip
    path = str(tmp_path / "ddos_distilbert_model.pth")
    ck.save_model(m, path)
    out = tmp_path / "preds.csv"
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-m", PKG, "predict", "--checkpoint", path, "--rows", "96", "--batch-size",
                        "32", "--out", str(out)], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    info = json.loads(r.stdout.strip().splitlines()[-1])
    assert info["rows"] == 96 and "f1" in info
    import pandas as pd
    df = pd.read_csv(out)
    assert list(df.columns) == ["row", "prob_ddos", "pred", "label"] and len(df) == 96
    assert ((df.prob_ddos >= 0) & (df.prob_ddos <= 1)).all()


@pytest.mark.gpu
def test_graphed_forward_matches_eager():
    from importlib import import_module
    models = import_module(f"{PKG}.models")
    engine = import_module(f"{PKG}.engine")
    m = models.DDoSClassifier(config=models.DistilBertConfig(n_layers=2), device="cuda", impl="hip", seed=2)
    m.eval()
    fwd = engine.GraphedForward(m)
    g = torch.Generator().manual_seed(0)
    for it in range(4):
        B, S = 16, 128
        lens = torch.randint(40 + 20 * (it % 2), 90, (B,), generator=g)
        mask = (torch.arange(S)[None] < lens[:, None]).long()
        ids = torch.randint(1000, 2000, (B, S), generator=g) * mask
        ids[:, 0] = 101
        ids, mask = ids.cuda(), mask.cuda()
        tok = int(lens.sum())
        a = fwd(ids, mask, tok).clone()
        with torch.no_grad():
            b = m(ids, mask, tokens=tok)
            c = m(ids, mask)  # padded path
        torch.cuda.synchronize()
        assert torch.equal(a, b)
        assert (a - c).abs().max().item() < 1e-2
    assert len(fwd.graphs) >= 2 and fwd.failed is None
