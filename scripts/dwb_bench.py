"""Isolated timing of the all-layer weight-gradient launch (ops/kernels.py linear_dw_batch) at
the packed bs32 x seq128 step's shapes (K = 2688 tokens, 6 layers x {qkv, o, lin1, lin2}),
with and without the fused Adam epilogue, per tile configuration."""
import sys
import time

import torch

sys.path.insert(0, ".")
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K  # noqa

T = int(sys.argv[1]) if len(sys.argv) > 1 else 2688
cfgs = [int(c) for c in (sys.argv[2] if len(sys.argv) > 2 else "8,1,12,4,21,15,0,10").split(",")]
g = torch.Generator(device="cuda").manual_seed(0)
shapes = [(2304, 768), (768, 768), (3072, 768), (768, 3072)] * 6
jobs, states = [], []
flops = 0
for M, N in shapes:
    dy = (torch.randn(T, M, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
    x = torch.randn(T, N, device="cuda", generator=g).to(torch.bfloat16)
    out = torch.empty(M, N, device="cuda")
    jobs.append((dy, x, out, False))
    states.append([torch.randn(M * N, device="cuda"), torch.zeros(M * N, device="cuda"),
                   torch.zeros(M * N, device="cuda"), torch.empty(M * N, device="cuda", dtype=torch.bfloat16)])
    flops += 2.0 * M * N * T
step = torch.ones(1, dtype=torch.int32, device="cuda")


def adam(outs, n_wT=0):
    st = []
    for s in states[:len(outs)]:
        st += s
    return st + [step], [2e-5, 0.9, 0.999, 1e-8, 0.0, 0.0]


for cfg in cfgs:
    for fused in (False, True):
        fn = (lambda: K.linear_dw_batch(jobs, adam=adam if fused else None, cfg=cfg))
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / n * 1e3
        print(f"cfg {cfg:2d} adam={int(fused)}  {us:8.1f} us  {flops / us / 1e6:7.1f} TF/s", flush=True)
