import sys, torch
sys.path.insert(0, ".")
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.models import DDoSClassifier, DistilBertConfig
sys.path.insert(0, "tests")
from test_prune_gpu import _batch
for mode in ("eval", "train_nodrop", "train"):
    for packed in (True, False):
        res = []
        for prune in (True, False):
            cfg = DistilBertConfig(n_layers=2)
            if mode == "train_nodrop":
                cfg.dropout = 0.0; cfg.attention_dropout = 0.0
            m = DDoSClassifier(config=cfg, device="cuda", impl="hip", seed=31)
            m.prune_last = prune
            if mode == "eval": m.eval()
            else:
                m.train()
                if mode == "train_nodrop": m.dropout.p = 0.0
            ids, mask, labels, tokens = _batch(32, 128, seed=800)
            m.rng.fill_(5)
            with torch.no_grad():
                z = m(ids, mask, tokens=tokens if packed else None)
            res.append(z.float())
        print(mode, "packed" if packed else "padded", (res[0] - res[1]).abs().max().item(), flush=True)
