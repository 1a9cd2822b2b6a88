"""Kernel-level comparison: split-K output LayerNorm + head_ln_bwd (two launches) vs the head fused
into the split-K LayerNorm epilogue (linear_ln_fwd_head): max differences of every output."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K  # noqa: E402


def main():
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(0)
    M, B, N, KK = 64, 32, 768, 3072
    bf = lambda *s, sc=1.0: (torch.randn(*s, generator=g) * sc).to(torch.bfloat16).to(dev)
    x, w, res = bf(M, KK), bf(N, KK, sc=0.03), bf(M, N)
    b = (torch.randn(N, generator=g) * 0.1).to(dev)
    gamma = (torch.randn(N, generator=g) * 0.2 + 1).to(dev)
    beta = (torch.randn(N, generator=g) * 0.1).to(dev)
    hW = (torch.randn(2, N, generator=g) * 0.05).to(dev)
    hb = torch.zeros(2, device=dev)
    labels = torch.randint(0, 2, (B,), generator=g).to(dev)
    seed = torch.tensor([5], dtype=torch.int32, device=dev)
    rm = torch.arange(M, dtype=torch.int32, device=dev) * 3
    for p, ph in ((0.0, 0.0), (0.1, 0.3)):
        thr, sc = K._drop(p)
        # A: LayerNorm (split-K) then the fused-head launch
        y, z, mean, rstd = K.linear_ln_fwd(x, w, b, res, gamma, beta, 1e-12, seed, 9, p, rm)
        dW, db = torch.zeros(2, N, device=dev), torch.zeros(2, device=dev)
        dg, dbt, dbi = (torch.zeros(N, device=dev) for _ in range(3))
        jobs = []
        logits, loss, dlog, dz, dx = K.head_ln_bwd(y, B, hW, hb, seed, 2, ph, labels, dW, db, False, None, z, gamma,
                                                   mean, rstd, 9, p, rm, dg, dbt, dbi, False, jobs)
        K.colsum_flush(jobs)
        # B: one launch
        dW2, db2 = torch.zeros(2, N, device=dev), torch.zeros(2, device=dev)
        dg2, dbt2, dbi2 = (torch.zeros(N, device=dev) for _ in range(3))
        jobs2 = []
        y2, z2, mean2, rstd2, (logits2, loss2, dz2, dx2) = K.linear_ln_fwd_head(
            x, w, b, res, gamma, beta, 1e-12, seed, 9, p, rm, hW, hb, 2, ph, labels, B, None, None, dW2, db2, False,
            dg2, dbt2, dbi2, False, jobs2)
        K.colsum_flush(jobs2)
        torch.cuda.synchronize()

        def d(a, c):
            a, c = a.float(), c.float()
            return f"max {((a - c).abs().max()).item():.3e} rel {((a - c).norm() / c.norm().clamp_min(1e-30)).item():.2e}"
        print(f"p {p} p_head {ph}: y equal {torch.equal(y, y2)} z equal {torch.equal(z, z2)} logits equal "
              f"{torch.equal(logits, logits2)} loss {loss.item():.8f} vs {loss2.item():.8f}")
        for nm, a, c in (("dz", dz2, dz), ("dx", dx2, dx), ("dW", dW2, dW), ("db", db2, db), ("dgamma", dg2, dg),
                         ("dbeta", dbt2, dbt), ("dbias", dbi2, dbi)):
            print(f"   {nm:7s} {d(a, c)}")


if __name__ == "__main__":
    main()
