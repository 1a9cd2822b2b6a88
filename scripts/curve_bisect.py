"""Bisect of the HIP-vs-fp32 loss-curve bias (tests/test_numerics_gpu.py test_loss_curve_parity_200_steps).

Round 3 found the HIP curve 1.3 % below the fp32 torch curve over 200 hard-profile steps, unchanged
with every HIP fast path off and with dropout off, while fp32 under bf16 autocast + bf16 storage
tracked fp32 within 0.0005.  The cause was in the fp32 ARM: on the GPU the torch path's word-
embedding rows went through the row-flag Adam (``adam_rows``), whose "has state" flags only the
HIP embedding backward sets -- so the fp32 reference never updated its 23.4 M word-embedding
parameters (engine/optim.py, fixed in round 4).

This script substitutes that one component between the arms: each path with its word-embedding
update on (fixed) or frozen (the round-3 reference arm's behaviour, emulated by restoring the
table after every step), two dropout streams each, and prints the 20-step window means, the mean
signed HIP - torch difference and the self-spread.  Usage: python scripts/curve_bisect.py
(BISECT_STEPS=200)."""
import gc
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.data import (  # noqa: E402
    DeviceLoader, build_client_data, generate_cicids2017)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.engine import (  # noqa: E402
    ArenaAdam, GraphedTrainStep, evaluate_model, make_step_fn)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.models import (  # noqa: E402
    DDoSClassifier)


def curve(impl, batches, test, counter0=0, freeze_word=False):
    m = DDoSClassifier(device="cuda", impl=impl, seed=8)
    opt = ArenaAdam(m, lr=2e-5)
    step = GraphedTrainStep(make_step_fn(m, opt), warmup=2, enabled=(impl == "hip"),
                            bucket=m.packed_rows if impl == "hip" else None)
    m.train()
    m.rng.fill_(counter0)
    m.torch_counter = counter0
    A = m.arena
    woff, V, D = m.word_embedding_span()
    wsl = slice(woff, woff + V * D)
    w0 = A.master[wsl].clone()
    moved = 0.0
    out = []
    for b in batches:
        out.append(step(b["input_ids"], b["attention_mask"], b["labels"],
                        b["n_tokens"] if impl == "hip" else None).clone())
        if freeze_word:  # the round-3 reference arm: word rows never updated
            with torch.no_grad():
                A.master[wsl].copy_(w0)
                A.shadow[wsl].copy_(w0.to(A.shadow.dtype))
    with torch.no_grad():
        moved = float((A.master[wsl] - w0).norm() / w0.norm())
    c = torch.stack(out).float().cpu().numpy()
    acc = evaluate_model(m, DeviceLoader(test, 64, device="cuda"))[0]
    del step, opt, m
    gc.collect()
    torch.cuda.empty_cache()
    return c, acc, moved


def main():
    n = int(os.environ.get("BISECT_STEPS", "200"))
    frame = generate_cicids2017(8000, seed=5, hard=True)
    cd = build_client_data(frame, 0, data_fraction=1.0, max_len=128)
    loader = DeviceLoader(cd.train, 32, shuffle=True, device="cuda", seed=3, drop_last=True)
    batches = []
    while len(batches) < n:
        batches.extend(loader)
    batches = batches[:n]
    W = n // 20
    runs = {}
    for impl in ("torch", "hip"):
        for frz in (False, True):
            for c0 in (0, 1 << 16):
                c, acc, moved = curve(impl, batches, cd.test, c0, frz)
                runs[(impl, frz, c0)] = (c.reshape(W, 20).mean(1), acc, moved)
                print(f"{impl:5s} word-rows {'frozen ' if frz else 'trained'} stream {c0:6d}: "
                      f"final acc {acc:6.2f} %  word-table moved {moved:.2e}  | "
                      + " ".join(f"{x:.3f}" for x in runs[(impl, frz, c0)][0]), flush=True)

    def cmp(name, a, b):
        # a, b: (impl, frozen) arms; both dropout streams; self-spread = the larger same-arm spread
        d = np.concatenate([runs[a + (c0,)][0] - runs[b + (c0,)][0] for c0 in (0, 1 << 16)])
        spread = np.maximum(np.abs(runs[a + (0,)][0] - runs[a + (1 << 16,)][0]),
                            np.abs(runs[b + (0,)][0] - runs[b + (1 << 16,)][0]))
        print(f"{name:44s} mean signed diff {d.mean():+.5f}  windows below {int((d < 0).sum()):2d}/{d.size}  "
              f"mean self-spread {spread.mean():.5f}  |bias|/spread {abs(d.mean()) / spread.mean():.2f}", flush=True)

    print("# substitution of ONE component (the word-embedding optimizer update) between the arms:")
    cmp("hip (trained) - torch (trained)   [fixed]", ("hip", False), ("torch", False))
    cmp("hip (trained) - torch (frozen)    [round 3]", ("hip", False), ("torch", True))
    cmp("hip (frozen)  - torch (frozen)", ("hip", True), ("torch", True))
    cmp("hip (frozen)  - torch (trained)", ("hip", True), ("torch", False))
    cmp("torch (frozen) - torch (trained)", ("torch", True), ("torch", False))


if __name__ == "__main__":
    main()
