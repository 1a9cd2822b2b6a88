"""|mean| / std of the LayerNorm input z per row at every block LayerNorm of the model's CPU fp32
path (random init, one bs8 synthetic batch): the regime of profiles/r6_ln_algebra_precision.txt.

  python scripts/ln_row_stats.py
"""
import os
import sys
from importlib import import_module

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
P = "detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd"
R = import_module(P + ".ops.reference")
models = import_module(P + ".models")
data = import_module(P + ".data")


def main():
    rec = []
    orig = R.add_ln_ref

    def hook(x, r, *a, **k):
        z = (x + r).float() if r is not None else x.float()
        rec.append((z.mean(-1).abs() / z.std(-1, unbiased=False)).flatten())
        return orig(x, r, *a, **k)

    R.add_ln_ref = hook
    torch.manual_seed(0)
    df = data.generate_cicids2017(400, seed=0)
    cd = data.build_client_data(df, 0, data_fraction=1.0, max_len=128)
    cpu = torch.device("cpu")
    model = models.DDoSClassifier(device=cpu)
    b = next(iter(data.DeviceLoader(cd.train, 8, device=cpu)))
    model.eval()
    with torch.no_grad():
        model(b["input_ids"], b["attention_mask"])
    R.add_ln_ref = orig
    for i, v in enumerate(rec):
        print(f"LayerNorm call {i}: |mean|/std per row  median {v.median():.3f}  p99 {v.quantile(0.99):.3f}  max {v.max():.3f}")


if __name__ == "__main__":
    main()
