"""Isolated timing of the NT GEMMs of the bs32 x seq128 packed step (M = 2688 rows): the LDS-DMA
kernels (gemm_kernel, picked per shape) against the direct-A kernels (gemm_da_kernel, 50: 128 x 64,
52: 128 x 128).  python scripts/da_bench.py [M]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as kn  # noqa: E402


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
    g = torch.Generator(device="cpu").manual_seed(0)

    def bf(*s, scale=1.0):
        return (torch.randn(*s, generator=g) * scale).to(torch.bfloat16).to("cuda")
    cases = []
    x768, x3072 = bf(M, 768), bf(M, 3072)
    wq, bq = bf(2304, 768, scale=0.03), torch.zeros(2304, device="cuda")
    w1, b1 = bf(3072, 768, scale=0.03), torch.zeros(3072, device="cuda")
    wo = bf(768, 768, scale=0.03)
    w2t = bf(3072, 768, scale=0.03)       # lin2's W^T [3072, 768] (FFN2 dX: dg = df W2)
    u = bf(M, 3072)
    w2 = w2t.t().contiguous()             # lin2's weight [768, 3072]
    cases.append(("qkv fwd   N=2304 K=768 ", lambda: kn.linear_fwd(x768, wq, bq), 2 * M * 2304 * 768))
    cases.append(("ffn1 fwd  N=3072 K=768 ", lambda: kn.linear_fwd(x768, w1, b1, gelu=True), 2 * M * 3072 * 768))
    cases.append(("ffn2 dX   N=3072 K=768 ", lambda: kn.linear_dx(x768, w2t.t(), gelu_u=u, wt=w2t), 2 * M * 3072 * 768))
    cases.append(("o dX      N=768  K=768 ", lambda: kn.linear_dx(x768, wo.t(), wt=wo), 2 * M * 768 * 768))
    cases.append(("o fwd     N=768  K=768 ", lambda: kn.linear_fwd(x768, wo, None), 2 * M * 768 * 768))
    cases.append(("lin2 fwd  N=768  K=3072", lambda: kn.linear_fwd(x3072, w2, None),
                  2 * M * 768 * 3072))
    for name, fn, fl in cases:
        line = f"{name}"
        for da in (-1, 50, 52):
            kn.ext().gemm_set_da(da)
            t = timed(fn)
            line += f"  da{da:3d} {t:7.2f} us {fl / t / 1e6:6.0f} TF/s"
        print(line, flush=True)
    kn.ext().gemm_set_da(-1)


if __name__ == "__main__" and not os.environ.get("DX_LAYOUTS"):
    main()


def dx_layouts():
    """The backward dX GEMMs on a W^T copy (NT, K-major B) vs on the weight itself (NN, MN-major B:
    no per-step transpose), LDS-DMA kernels and direct-A kernels; plus the LayerNorm-fused dX."""
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 2688
    g = torch.Generator(device="cpu").manual_seed(1)

    def bf(*s, scale=1.0):
        return (torch.randn(*s, generator=g) * scale).to(torch.bfloat16).to("cuda")
    # (name, K = dy width, N = dx width, epi): W is [K, N] (the Linear weight [out = K, in = N])
    shapes = [("qkv dX  ", 2304, 768), ("lin1 dX ", 3072, 768), ("lin2 dX ", 768, 3072), ("o dX    ", 768, 768)]
    for name, K, N in shapes:
        dy, w = bf(M, K), bf(K, N, scale=0.03)
        wt = w.t().contiguous()
        res = bf(M, N)
        line = f"{name} N={N:4d} K={K:4d}"
        for da in (-1, 50):
            kn.ext().gemm_set_da(da)
            t_nt = timed(lambda: kn.linear_dx(dy, w, res=res, wt=wt))
            t_nn = timed(lambda: kn.linear_dx(dy, w, res=res))
            line += f" | da{da:3d} NT {t_nt:6.2f} NN {t_nn:6.2f} us"
        kn.ext().gemm_set_da(-1)
        print(line, flush=True)
    # LayerNorm-fused backward (N = 768): W^T (K-major) vs W (MN-major), LDS-DMA cfg 24 and direct-A 50
    D = 768
    gamma = torch.ones(D, device="cuda")
    mean, rstd = torch.zeros(M, device="cuda"), torch.ones(M, device="cuda")
    seed = torch.tensor([3], dtype=torch.int32, device="cuda")
    stats, cnt, err = kn._ln_state(torch.device("cuda"), M, D)
    cp = torch.empty(((M + 63) // 64) * 3 * D, device="cuda")
    thr, sc = kn._drop(0.1)
    site = [kn.LN_XSITES]

    def xs():
        site[0] += 1
        if site[0] >= kn.LN_XSITES:
            kn.ln_epoch_advance("cuda")
            site[0] = 0
        return site[0]
    for K in (3072, 2304):
        a, w = bf(M, K, scale=0.5), bf(K, D, scale=0.03)
        wt = w.t().contiguous()
        z, res = bf(M, D), bf(M, D)
        dz, dx = torch.empty_like(z), torch.empty_like(z)
        line = f"ln bwd K={K}"
        for cfg in (24, 50):
            for bmn in (False, True):
                B = w if bmn else wt
                t = timed(lambda: kn.ext().gemm_ln(True, a, B, dz, None, res, gamma, None, mean, rstd, z, dx, cp,
                                                   stats, cnt, err, 0.0, seed, 9, thr, sc, None, cfg, xs(), bmn))
                line += f" | cfg{cfg} {'W ' if bmn else 'WT'} {t:6.2f}"
        print(line, flush=True)
    torch.cuda.synchronize()
    print("err flag", int(err.item()))


if __name__ == "__main__" and os.environ.get("DX_LAYOUTS"):
    dx_layouts()
