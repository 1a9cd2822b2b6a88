"""Split-K probe for the grouped weight-gradient GEMMs (TN, K = packed tokens).

The default plan only doubles the split count while K / (2 * splits) stays a
multiple of 64, so at T = 2688 it stops at 2 (o+qkv) / 1 (ffn).  This times the
grouped dW launches with split counts that divide T / 64 (1, 2, 3, 6, 7 at
T = 2688) for a few tile configurations, slab reduce included (non-deferred),
and checks against torch fp32.

usage: python scripts/dw_split_probe.py [T=2688]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops._ext import ext

T = int(sys.argv[1]) if len(sys.argv) > 1 else 2688
g = torch.Generator(device="cuda").manual_seed(0)


def rnd(*s, scale=1.0):
    return ((torch.rand(*s, device="cuda", generator=g) * 2 - 1) * scale).to(torch.bfloat16)


def timeit(fn, iters=40):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


shapes = {"qkv": (2304, 768), "o": (768, 768), "ffn1": (3072, 768), "ffn2": (768, 3072)}
data = {k: (rnd(T, n), rnd(T, kd)) for k, (n, kd) in shapes.items()}
splits_opts = [s for s in (1, 2, 3, 4, 6, 7, 8) if T % (64 * s) == 0]
for a, b in (("ffn2", "ffn1"), ("o", "qkv")):
    (dya, xa), (dyb, xb) = data[a], data[b]
    oa = torch.empty(dya.shape[1], xa.shape[1], device="cuda")
    ob = torch.empty(dyb.shape[1], xb.shape[1], device="cuda")
    ref = torch.cat([(dya.float().t() @ xa.float()).flatten(), (dyb.float().t() @ xb.float()).flatten()])
    macs = T * (oa.numel() + ob.numel())

    def fn():
        K.linear_dw2(dya, xa, oa, dyb, xb, ob)
        return torch.cat([oa.flatten(), ob.flatten()])

    for cfg in (8, 1, 19, 13, 0, 2):
        for sp in splits_opts:
            ext().gemm_set_cfg(2, cfg, sp)
            try:
                out = fn()
                torch.cuda.synchronize()
            except RuntimeError:
                continue
            err = ((out - ref).abs().max() / ref.abs().max()).item()
            us = timeit(fn)
            print(f"{a}+{b}.dW cfg={cfg:2d} splits={sp}  {us:7.1f} us  {2 * macs / us / 1e6:5.0f} TF  err={err:.1e}"
                  f"{'' if err < 2e-2 else '  BAD'}", flush=True)
    ext().gemm_set_cfg(2, -1, -1)
    print(f"{a}+{b}.dW default          {timeit(fn):7.1f} us", flush=True)
