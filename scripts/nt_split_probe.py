"""Probe: NT GEMM (M=T, N=768, K in {2304, 3072}) as fp32 split-K partials, per config and
split count, vs the plain bf16 NT kernel -- does splitting K buy back the idle CUs?
usage: python scripts/nt_split_probe.py [T=2688]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops._ext import ext

T = int(sys.argv[1]) if len(sys.argv) > 1 else 2688


def timeit(fn, iters=30):
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


g = torch.Generator(device="cuda").manual_seed(0)
for Kd in (2304, 3072):
    N = 768
    x = (torch.randn(T, Kd, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, Kd, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    y = torch.empty(T, N, dtype=torch.bfloat16, device="cuda")
    ref = x.float() @ w.float().t()
    base = timeit(lambda: ext().gemm(0, 0, x, w, y, None, None, None, None, False))
    print(f"K={Kd}: plain bf16 NT default cfg {base:6.1f} us", flush=True)
    ws = torch.empty(8 * T * N, device="cuda")
    for cfg in (0, 1, 8, 10, 17):
        for sp in (2, 3, 4):
            if Kd % (sp * 64):
                continue
            ext().gemm_set_cfg(0, cfg, -1)
            ext().gemm_set_cfg(2, -1, sp)  # FD_GEMM_SPLITS (shared override)
            out = torch.empty(T, N, dtype=torch.bfloat16, device="cuda")  # unused (partials go to ws)
            try:
                ext().gemm(0, 5, x, w, out, None, None, None, ws, False)
            except RuntimeError as e:
                print(f"  cfg={cfg} splits={sp}: {e}")
                continue
            torch.cuda.synchronize()
            tot = ws[:sp * T * N].view(sp, T, N).sum(0)
            err = ((tot - ref).abs().max() / ref.abs().max()).item()
            us = timeit(lambda: ext().gemm(0, 5, x, w, out, None, None, None, ws, False))
            red = timeit(lambda: ws[:sp * T * N].view(sp, T, N).sum(0))
            print(f"  cfg={cfg:2d} splits={sp}: {us:6.1f} us partials (+ torch reduce {red:5.1f} us)  err={err:.1e}",
                  flush=True)
    ext().gemm_set_cfg(0, -1, -1)
    ext().gemm_set_cfg(2, -1, -1)
