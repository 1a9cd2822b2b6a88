"""Bisect the HIP-vs-fp32 loss-curve bias (tests/test_numerics_gpu.py test_loss_curve_parity_200_steps):
the same 200 hard-profile batches, the same dropout stream, HIP variants with one fast path off at a
time, against the fp32 torch path.  Prints 20-step window means and the mean signed HIP - torch."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.data import (  # noqa: E402
    DeviceLoader, build_client_data, generate_cicids2017)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.engine import (  # noqa: E402
    ArenaAdam, GraphedTrainStep, make_step_fn)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.models import (  # noqa: E402
    DDoSClassifier, DistilBertConfig)


def curve(impl, batches, graph=True, packed=True, prune=True, fuse_ln=True, fused_adam=True, nodrop=False,
          steps=200, autocast=False):
    cfg = DistilBertConfig(dropout=0.0, attention_dropout=0.0) if nodrop else DistilBertConfig()
    m = DDoSClassifier(config=cfg, device="cuda", impl=impl, seed=8, **({"head_dropout": 0.0} if nodrop else {}))
    if impl == "hip":
        m.prune_last, m.fuse_ln = prune, fuse_ln
    opt = ArenaAdam(m, lr=2e-5, fuse_dw=fused_adam)
    use_tok = impl == "hip" and packed
    step = GraphedTrainStep(make_step_fn(m, opt), warmup=2, enabled=(impl == "hip" and graph),
                            bucket=m.packed_rows if use_tok else None)
    m.train()
    m.rng.fill_(0)
    m.torch_counter = 0
    out = []
    for b in batches[:steps]:
        # autocast: the fp32 torch path with its matmuls in bf16 (fp32 accumulate) -- a control for
        # "is the HIP-vs-fp32 difference the bf16 arithmetic itself?"
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
            out.append(step(b["input_ids"], b["attention_mask"], b["labels"], b["n_tokens"] if use_tok else None).clone())
    c = torch.stack(out).float().cpu().numpy()
    del step, opt, m
    torch.cuda.empty_cache()
    return c


def main():
    frame = generate_cicids2017(8000, seed=5, hard=True)
    cd = build_client_data(frame, 0, data_fraction=1.0, max_len=128)
    loader = DeviceLoader(cd.train, 32, shuffle=True, device="cuda", seed=3, drop_last=True)
    batches = []
    while len(batches) < 200:
        batches.extend(loader)
    batches = batches[:200]
    ref = {False: curve("torch", batches), True: curve("torch", batches, nodrop=True)}
    variants = [("hip default", {}), ("eager (no graph)", {"graph": False}), ("padded", {"packed": False}),
                ("no [CLS] pruning", {"prune": False}), ("unfused LN", {"fuse_ln": False}),
                ("unfused Adam", {"fused_adam": False}),
                ("all off", {"graph": False, "packed": False, "prune": False, "fuse_ln": False, "fused_adam": False}),
                ("dropout off", {"nodrop": True})]
    if os.environ.get("BISECT_QUICK"):
        variants = [variants[0], variants[-1]]
    for name, kw in variants:
        c = curve("hip", batches, **kw)
        r = ref[kw.get("nodrop", False)]
        wh, wr = c.reshape(10, 20).mean(1), r.reshape(10, 20).mean(1)
        d = wh - wr
        print(f"{name:18s} mean(hip-torch) {d.mean():+.5f}  windows hip<torch {int((d < 0).sum()):2d}/10  "
              f"last3 {d[-3:].mean():+.5f}  | hip {' '.join(f'{x:.3f}' for x in wh)}", flush=True)
    from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import reference as REF
    for nodrop in (False, True):
        REF.BF16_STORAGE = True  # + every tensor the HIP path stores in bf16 rounded to bf16
        c = curve("torch", batches, nodrop=nodrop, autocast=True)
        REF.BF16_STORAGE = False
        r = ref[nodrop]
        wh, wr = c.reshape(10, 20).mean(1), r.reshape(10, 20).mean(1)
        d = wh - wr
        print(f"{'torch bf16 storage' + (' nodrop' if nodrop else ''):18s} mean(bf16-fp32) {d.mean():+.5f}  windows "
              f"bf16<fp32 {int((d < 0).sum()):2d}/10  last3 {d[-3:].mean():+.5f}  | {' '.join(f'{x:.3f}' for x in wh)}",
              flush=True)
    for nodrop in (False, True):
        c = curve("torch", batches, nodrop=nodrop, autocast=True)
        r = ref[nodrop]
        wh, wr = c.reshape(10, 20).mean(1), r.reshape(10, 20).mean(1)
        d = wh - wr
        print(f"{'torch bf16 autocast' + (' nodrop' if nodrop else ''):18s} mean(bf16-fp32) {d.mean():+.5f}  windows "
              f"bf16<fp32 {int((d < 0).sum()):2d}/10  last3 {d[-3:].mean():+.5f}  | {' '.join(f'{x:.3f}' for x in wh)}",
              flush=True)
    for k, r in ref.items():
        print(f"torch {'nodrop' if k else 'drop  '}        {' '.join(f'{x:.3f}' for x in r.reshape(10, 20).mean(1))}")


if __name__ == "__main__":
    main()
