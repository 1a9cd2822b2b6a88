"""Isolated timing of the LayerNorm-fused N = 768 GEMMs vs GEMM + separate LN kernel.

    python scripts/ln_fused_bench.py [M] [cfgs]      e.g.  2688 24,0,18,13
Per configuration (FD_GEMM_LN_CFG-equivalent cfg argument) the forward shapes of out_lin
(K = 768) and lin2 (K = 3072) and the backward shapes of the lin1 dX (K = 3072) and qkv dX
(K = 2304) GEMMs, bs32 x seq128 packed rows.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as kn  # noqa: E402
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops._ext import ext  # noqa: E402

D = 768


def timed(fn, iters=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / iters


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 2688
    cfgs = [int(c) for c in (sys.argv[2] if len(sys.argv) > 2 else "24").split(",")]
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(0)

    def bf(*s, scale=1.0):
        return (torch.randn(*s, generator=g) * scale).to(torch.bfloat16).to(dev)
    gamma, beta = torch.ones(D, device=dev), torch.zeros(D, device=dev)
    seed = torch.tensor([3], dtype=torch.int32, device=dev)
    res = bf(M, D)
    y, z = torch.empty(M, D, dtype=torch.bfloat16, device=dev), torch.empty(M, D, dtype=torch.bfloat16, device=dev)
    mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
    stats, cnt, err = kn._ln_state(torch.device(dev), M, D)
    cp = torch.empty(((M + 63) // 64) * 3 * D, device=dev)
    thr, sc = kn._drop(0.1)
    site = [kn.LN_XSITES]

    def xs():  # a fresh exchange call site per launch (a new epoch every LN_XSITES launches)
        site[0] += 1
        if site[0] >= kn.LN_XSITES:
            kn.ln_epoch_advance(dev)
            site[0] = 0
        return site[0]
    for K in (768, 3072):
        x, w, b = bf(M, K), bf(D, K, scale=0.03), torch.zeros(D, device=dev)
        t_ref = timed(lambda: kn.ln_fwd(kn.linear_fwd(x, w, b), res, gamma, beta, 1e-12, seed, 9, 0.1))
        line = f"fwd K={K:5d}  gemm+ln {t_ref:7.1f} us"
        for c in cfgs:
            t = timed(lambda: ext().gemm_ln(False, x, w, y, b, res, gamma, beta, mean, rstd, z, None, None, stats, cnt,
                                            err, 1e-12, seed, 9, thr, sc, None, c, xs()))
            line += f"   cfg{c} {t:7.1f}"
        print(line, flush=True)
    for K in (3072, 2304):
        a, wt = bf(M, K, scale=0.5), bf(D, K, scale=0.03)
        dg, db, dbi = (torch.empty(D, device=dev) for _ in range(3))
        dz, dx = torch.empty_like(y), torch.empty_like(y)
        t_ref = timed(lambda: kn.ln_bwd(kn.linear_dx(a, wt.t().contiguous(), res=res), z, None, gamma, mean, rstd, dg, db,
                                        dbi, seed, 9, 0.1, zin=True, jobs=[]))
        line = f"bwd K={K:5d}  gemm+ln {t_ref:7.1f} us"
        for c in cfgs:
            t = timed(lambda: ext().gemm_ln(True, a, wt, dz, None, res, gamma, None, mean, rstd, z, dx, cp, stats, cnt,
                                            err, 0.0, seed, 9, thr, sc, None, c, xs()))
            line += f"   cfg{c} {t:7.1f}"
        print(line, flush=True)
    torch.cuda.synchronize()
    print("err flag", int(err.item()), "epoch", int(cnt[0].item()))


if __name__ == "__main__":
    main()
