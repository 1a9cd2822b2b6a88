"""Parity with the model the reference actually runs: HF ``transformers.DistilBertModel``
(/root/reference/client1.py:56,61-64) + Dropout(0.3) + Linear(768, 2).

Our ``state_dict()`` (102 keys) loads strict into the HF module tree; in eval mode the
pure-torch path (``impl="torch"``, the CPU execution path and the oracle every HIP kernel test
compares against) must give the HF logits and the HF parameter gradients of the CE loss.
CPU-only (transformers 5.15 is importable here; no network: random init, no pretrained weights).
"""
import pytest
import torch

from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.models import (
    DDoSClassifier, DistilBertConfig)

transformers = pytest.importorskip("transformers")


class _HFClassifier(torch.nn.Module):
    """The reference DDoSClassifier (client1.py:53-65) on a config instead of a pretrained dir."""

    def __init__(self):
        super().__init__()
        cfg = transformers.DistilBertConfig()
        cfg._attn_implementation = "eager"
        self.distilbert = transformers.DistilBertModel(cfg)
        self.dropout = torch.nn.Dropout(0.3)
        self.classifier = torch.nn.Linear(768, 2)

    def forward(self, input_ids, attention_mask):
        out = self.distilbert(input_ids=input_ids, attention_mask=attention_mask)
        return self.classifier(self.dropout(out[0][:, 0, :]))


def _batch(B=4, S=48, seed=0):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(1000, 30000, (B, S), generator=g)
    lens = torch.randint(S // 2, S + 1, (B,), generator=g)
    lens[0] = S
    mask = (torch.arange(S)[None] < lens[:, None]).long()
    ids = ids * mask
    ids[:, 0] = 101
    return ids, mask, torch.randint(0, 2, (B,), generator=g)


@pytest.fixture(scope="module")
def pair():
    torch.manual_seed(0)
    ours = DDoSClassifier(config=DistilBertConfig(), impl="torch", seed=5)
    hf = _HFClassifier()
    missing = hf.load_state_dict(ours.state_dict(), strict=True)
    assert not missing.missing_keys and not missing.unexpected_keys
    ours.eval()
    hf.eval()
    return ours, hf


def test_state_dict_keys_shapes_match_hf(pair):
    ours, hf = pair
    a, b = ours.state_dict(), hf.state_dict()
    assert list(a.keys()) == [k for k in b.keys()]  # same 102 keys in the same order
    assert all(a[k].shape == b[k].shape and a[k].dtype == b[k].dtype == torch.float32 for k in a)


def test_logits_match_hf(pair):
    ours, hf = pair
    ids, mask, _ = _batch()
    with torch.no_grad():
        za = ours(ids, mask)
        zb = hf(ids, mask)
    assert (za - zb).abs().max().item() <= 1e-5, (za - zb).abs().max().item()


def test_gradients_match_hf(pair):
    ours, hf = pair
    ids, mask, labels = _batch(seed=1)
    ours.zero_grad()
    hf.zero_grad(set_to_none=True)
    crit = torch.nn.CrossEntropyLoss()
    crit(ours(ids, mask), labels).backward()
    crit(hf(ids, mask), labels).backward()
    hp = dict(hf.named_parameters())
    worst = 0.0
    for name, p in ours.named_parameters():
        ga, gb = p.grad, hp[name].grad
        assert gb is not None, name
        den = gb.norm().item()
        if name.endswith("k_lin.bias"):
            # exactly zero in exact arithmetic (a key bias shifts every score of a query by the
            # same q.b_k, which softmax ignores): both sides are rounding noise
            assert ga.norm().item() < 1e-6 and den < 1e-6, (name, ga.norm().item(), den)
            continue
        err = (ga - gb).norm().item() / max(den, 1e-12)
        if den > 1e-10:
            worst = max(worst, err)
            assert err <= 1e-4, (name, err)
    assert worst <= 1e-4
