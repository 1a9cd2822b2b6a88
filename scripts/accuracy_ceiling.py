"""How high can a strong tabular model get on the synthetic generator's profiles, on the same 10
text-template features the model reads (data/featurize.py TEXT_FIELDS)?  Gradient-boosted trees
(sklearn HistGradientBoostingClassifier) on the full 225,745-row file (80 / 20) and on client-sized
10 % samples (60 / 20 / 20, seeds 42 + k) -- a reference point for the federated DistilBERT's
accuracy per profile.  CPU only, seconds.

    python scripts/accuracy_ceiling.py
"""
import sys

import numpy as np
from sklearn.ensemble import HistGradientBoostingClassifier

sys.path.insert(0, ".")
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.data import (  # noqa
    featurize as fz, synthetic as syn)


def xy(df):
    X = df[fz.FEATURE_COLUMNS].replace([np.inf, -np.inf], np.nan).astype(float)
    X = X.fillna(X.mean())
    lab = df[" Label"] if " Label" in df else df["Label"]
    return X.values, lab.astype(str).str.strip().ne("BENIGN").astype(int).values


def main():
    for prof in ("default", "calibrated"):
        X, y = xy(syn.generate_cicids2017(225_745, seed=0, profile=prof))
        n = len(y)
        idx = np.random.default_rng(42).permutation(n)
        tr, te = idx[: int(0.8 * n)], idx[int(0.8 * n):]
        full = HistGradientBoostingClassifier(max_iter=400, max_leaf_nodes=63, random_state=0).fit(X[tr], y[tr])
        accs = []
        for k in range(8):
            s = np.random.default_rng(42 + k).choice(n, n // 10, replace=False)
            a, b = int(0.6 * len(s)), int(0.8 * len(s))
            m = HistGradientBoostingClassifier(max_iter=400, max_leaf_nodes=63, random_state=0).fit(X[s[:a]], y[s[:a]])
            accs.append((m.predict(X[s[b:]]) == y[s[b:]]).mean())
        print(f"{prof}: GBDT on 180k rows -> held-out {100 * (full.predict(X[te]) == y[te]).mean():.3f} %; "
              f"client-sized (13.5k train, 8 samples) -> {100 * np.mean(accs):.3f} % "
              f"(min {100 * min(accs):.3f}, max {100 * max(accs):.3f})")


if __name__ == "__main__":
    main()
