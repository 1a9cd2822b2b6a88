"""Per-parameter gradient agreement of the pruned step's head inside the output-LayerNorm split-K
epilogue (FD_HEAD_IN_SK) against the separate fused-head launch (head_ln_bwd): prints the worst
relative differences (summation-order level expected)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.models import (  # noqa: E402
    DDoSClassifier, DistilBertConfig)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K  # noqa: E402


def batch(B, S, seed, empty=None):
    gen = torch.Generator().manual_seed(seed)
    ids = torch.randint(1000, 2000, (B, S), generator=gen)
    lens = torch.randint(60, 85, (B,), generator=gen)
    if empty is not None:
        lens[empty] = 0
    mask = (torch.arange(S)[None] < lens[:, None]).long()
    ids = ids * mask
    ids[:, 0] = 101
    if empty is not None:
        ids[empty] = 0
    labels = torch.randint(0, 2, (B,), generator=gen)
    return ids.cuda(), mask.cuda(), labels.cuda(), int(lens.sum())


def run(in_sk, B, empty, kd, packed=True):
    K.HEAD_IN_SK = in_sk
    m = DDoSClassifier(config=DistilBertConfig(n_layers=3), device="cuda", impl="hip", seed=43)
    m.train()
    ids, mask, labels, tokens = batch(B, 128, 812, empty)
    t = None
    if kd:
        g = torch.Generator(device="cuda").manual_seed(4)
        t = (torch.randn(B, 2, device="cuda", generator=g), 2.0, 0.9)
    m.zero_grad()
    m.rng.fill_(7)
    loss, logits = m.forward_loss(ids, mask, labels, tokens=tokens if packed else None, kd=t, unit_backward=True)
    loss.backward(K.unit_grad("cuda"))
    torch.cuda.synchronize()
    return loss.item(), logits.clone(), {k: m.dense_grad(k).clone() for k in m.state_dict()}


def worst(a, b):
    errs = []
    for k in b[2]:
        n = b[2][k].float().norm().item()
        if n > 0 and "k_lin.bias" not in k:  # (k_lin.bias: zero up to rounding noise)
            errs.append(((a[2][k] - b[2][k]).float().norm().item() / n, k))
    return max(errs)


for B, empty, kd, packed in ((32, None, False, True), (16, None, False, False)):
    a1, a2 = run(True, B, empty, kd, packed), run(True, B, empty, kd, packed)
    b1, b2 = run(False, B, empty, kd, packed), run(False, B, empty, kd, packed)
    print(f"repeat in_sk {worst(a1, a2)}  repeat fold {worst(b1, b2)}  in_sk vs fold {worst(a1, b1)}")

for B, empty, kd, packed in ((32, None, False, True), (20, 3, False, True), (16, None, False, False), (32, None, True, True)):
    a, b = run(True, B, empty, kd, packed), run(False, B, empty, kd, packed)
    print(f"B={B} empty={empty} kd={kd} packed={packed}: loss {a[0]:.7f} vs {b[0]:.7f}, logits equal {torch.equal(a[1], b[1])}")
    errs = []
    for k in b[2]:
        n = b[2][k].float().norm().item()
        if n > 0:
            errs.append(((a[2][k] - b[2][k]).float().norm().item() / n, k))
    if B == 32 and not kd:
        for e, k in errs:  # (state_dict order)
            print(f"   {e:.2e}  {k}")
    errs.sort(reverse=True)
    for e, k in errs[:6]:
        print(f"   {e:.2e}  {k}")
