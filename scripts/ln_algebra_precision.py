"""Precision of the consumer-side ("algebraic") LayerNorm the round-5 review proposed
(docs/ARCHITECTURE.md section 9 "Why the LayerNorm rendezvous stays", route (b)),
measured against what the LayerNorm-fused GEMMs do now.

The consumer of h = LN(z) (the next GEMM, out = h W^T) can skip the producer's LayerNorm by
    out = rstd * (z (gamma o W)^T - mean * (W gamma)) + W beta
with per-row (mean, rstd) merged from the producer's column partials.  Its operands are the raw
residual sum z and a per-step weight copy gamma o W, both in bf16 on the MFMA path.  Current path:
the producer normalises in fp32 and stores h in bf16; the GEMM multiplies bf16(h) by bf16(W).

Rows are z = mu + sigma * N(0, 1) (+ optional outlier columns, as trained transformers show), for a
sweep of |mu| / sigma.  Errors are the max relative error over the output (normalised by the
output's rms) against an fp64 reference.  CPU only; prints a table (profiles/r6_ln_algebra_precision.txt).

  python scripts/ln_algebra_precision.py
"""
from __future__ import annotations

import torch


def bf(x: torch.Tensor) -> torch.Tensor:
    return x.to(torch.bfloat16).to(torch.float32)


def run(ratio: float, outliers: bool, M: int = 1024, D: int = 768, N: int = 768, seed: int = 0):
    g = torch.Generator().manual_seed(seed)
    sigma = 1.0
    z = ratio * sigma * (1.0 + 0.1 * torch.randn(M, 1, generator=g, dtype=torch.float64)) \
        + sigma * torch.randn(M, D, generator=g, dtype=torch.float64)
    if outliers:  # a few large feature dimensions, as in trained BERT-family hidden states
        z[:, :4] += 20.0 * sigma * torch.randn(1, 4, generator=g, dtype=torch.float64)
    # z is exact here (fp64); the current route normalises the producer's fp32 accumulators, the
    # algebraic one needs z in memory: bf16 (what a GEMM epilogue writes) or fp32 (twice the bytes)
    gamma = 1.0 + 0.1 * torch.randn(D, generator=g, dtype=torch.float64)
    beta = 0.1 * torch.randn(D, generator=g, dtype=torch.float64)
    W = bf((torch.randn(N, D, generator=g, dtype=torch.float64) * 0.02).float()).double()
    eps = 1e-12
    mean = z.mean(1, keepdim=True)
    rstd = (z.var(1, unbiased=False, keepdim=True) + eps).rsqrt()
    ref = ((z - mean) * rstd * gamma + beta) @ W.T  # fp64 reference

    # current: fp32 LayerNorm in the producer, bf16 h, bf16 x bf16 GEMM with fp32 accumulation
    z32 = z.float()
    m32 = z32.mean(1, keepdim=True)
    r32 = (z32.var(1, unbiased=False, keepdim=True) + eps).rsqrt()
    h = bf((z32 - m32) * r32 * gamma.float() + beta.float())
    cur = h @ W.float().T

    # algebraic: z (bf16 on the MFMA path) times bf16 (gamma o W), fp32 accumulation, fp32 correction
    # terms; (mean, rstd) from the producer's fp32 partials (exact here)
    Wg = bf((W * gamma).float())
    rowWg = Wg.sum(1)  # W gamma (fp32 sum of the bf16 copy the GEMM uses)
    Wb = (W.float() @ beta.float())
    alg = r32 * (bf(z32) @ Wg.T - m32 * rowWg) + Wb
    # route (a): the consumer normalises its A operand in fp32 on the operand path, then casts to bf16 --
    # from z stored in bf16 (the producer's output width) or in fp32 (twice the bytes)
    ln = lambda zz: bf((zz - m32) * r32 * gamma.float() + beta.float())
    a_bf = ln(bf(z32)) @ W.float().T
    a_f32 = ln(z32) @ W.float().T

    rms = ref.pow(2).mean().sqrt()
    err = lambda o: ((o.double() - ref).abs().max() / rms).item()
    return err(cur), err(a_bf), err(a_f32), err(alg)


def main():
    print("max |out - ref| / rms(ref) against fp64 (x cur: the error over the current path's)")
    print("  current : fp32 LayerNorm of the producer's fp32 z, bf16 h, bf16 x bf16 GEMM (fp32 accumulation)")
    print("  (a) bf16: z stored in bf16, the consumer normalises it on its A-operand path")
    print("  (a) f32 : z stored in fp32 (2x the bytes), the consumer normalises it on its A-operand path")
    print("  (b)     : bf16 z x bf16 (gamma o W), minus mean (W gamma), times rstd, plus W beta")
    print(f"{'|mu|/sigma':>10} {'outliers':>8} {'current':>9} {'(a) bf16':>9} {'x cur':>6} {'(a) f32':>9} {'x cur':>6}"
          f" {'(b)':>9} {'x cur':>6}")
    for outliers in (False, True):
        for ratio in (0.0, 0.5, 2.0, 8.0, 32.0):
            c, abf, af, b = run(ratio, outliers)
            print(f"{ratio:>10.1f} {str(outliers):>8} {c:>9.2e} {abf:>9.2e} {abf / c:>6.1f} {af:>9.2e} {af / c:>6.1f}"
                  f" {b:>9.2e} {b / c:>6.1f}")


if __name__ == "__main__":
    main()
