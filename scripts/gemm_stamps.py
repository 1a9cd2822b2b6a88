"""Phase timing of the one-round GEMMs from in-kernel wall-clock stamps (diagnostic build).

    FD_BUILD_TAG=stamps FD_SO_OUT=ab/stamps.so FD_HIP_EXTRA_FLAGS=-DFD_GEMM_STAMPS=1 \
        python -m <pkg>._build            # (CPU, once)
    FD_SO_OUT=ab/stamps.so python scripts/gemm_stamps.py [M]

Per call (bs32 packed shapes): the LayerNorm-fused forward / backward GEMMs and the plain NT GEMMs
of the step.  Stamps (gemm.hip FD_STAMP, 100 MHz = 10 ns): 0 entry, 1 first K tile landed, 2 K loop
done, 3 LN statistics published, 4 row-block rendezvous done, 5 exit.  Printed per phase: the
median / max over blocks (us), the spread of block starts, and how many blocks shared a CU.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as kn  # noqa: E402
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops._ext import ext  # noqa: E402

D = 768


def report(name, nblocks, ln):
    st = torch.zeros(nblocks, 8, dtype=torch.int64)
    n = ext().gemm_stamps(st)
    if n < 0:
        print("not a stamps build")
        sys.exit(1)
    t = st[:, :6].double() / 100.0  # us
    t0 = t[:, 0].min()
    t = t - t0
    hw = st[:, 7]
    cu = ((hw >> 32) << 8) | ((hw >> 8) & 0xff)
    _, counts = torch.unique(cu, return_counts=True)

    def q(x):
        return f"{x.median().item():6.2f}/{x.max().item():6.2f}"
    line = (f"{name:26s} blocks {nblocks:4d} CUs {len(counts):3d} (max {counts.max().item()}/CU) "
            f"start {q(t[:, 0])} | prolog {q(t[:, 1] - t[:, 0])} | kloop {q(t[:, 2] - t[:, 1])}")
    if ln:
        line += f" | epi1 {q(t[:, 3] - t[:, 2])} | wait {q(t[:, 4] - t[:, 3])} | epi2 {q(t[:, 5] - t[:, 4])}"
    else:
        line += f" | epi {q(t[:, 5] - t[:, 2])}"
    line += f" | end {q(t[:, 5])}"
    print(line, flush=True)


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 2688
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

    def xs():
        site[0] += 1
        if site[0] >= kn.LN_XSITES - 1:  # (site LN_XSITES - 1 is never a valid call site)
            kn.ln_epoch_advance(dev)
            site[0] = 0
        return site[0]
    nb_ln = ((M + 127) // 128) * (D // 64)
    xbuf = kn.workspace(torch.device(dev), "ln2_xbuf", 128 * 2 * 16384)
    for rep in range(2):
        # two-K-half tiles (ln2: K >= 2048 with the exchange buffer) and the one-pass kernel;
        # ln2 stamps: 2 = this block's half of the K loop done, 3 = partials traded + statistics published
        for ln2 in (True, False):
            xb = xbuf if ln2 else None
            tg = "ln2" if ln2 else "ln"
            for K in (768, 3072):
                x, w, b = bf(M, K), bf(D, K, scale=0.03), torch.zeros(D, device=dev)
                for _ in range(20):
                    ext().gemm_ln(False, x, w, y, b, res, gamma, beta, mean, rstd, z, None, None, stats, cnt, err,
                                  1e-12, seed, 9, thr, sc, None, -1, xs(), False, xb)
                torch.cuda.synchronize()
                report(f"{tg} fwd K={K}", nb_ln, True)
            for K in (3072, 2304):
                a, wt = bf(M, K, scale=0.5), bf(D, K, scale=0.03)
                w_mn = wt.t().contiguous()  # W [K][N]: the model's dX GEMMs read the weight MN-major
                dz, dx = torch.empty_like(y), torch.empty_like(y)
                for b_mn, B, tag in ((True, w_mn, "NN"), (False, wt, "NT")):
                    for _ in range(20):
                        ext().gemm_ln(True, a, B, dz, None, res, gamma, None, mean, rstd, z, dx, cp, stats, cnt, err,
                                      0.0, seed, 9, thr, sc, None, -1, xs(), b_mn, xb)
                    torch.cuda.synchronize()
                    report(f"{tg} bwd {tag} K={K}", nb_ln, True)
        for (N, K, epi, nm) in ((768, 768, 0, "o dX"), (2304, 768, 1, "qkv fwd"), (3072, 768, 2, "ffn1 fwd")):
            x, w, b = bf(M, K), bf(N, K, scale=0.03), torch.zeros(N, device=dev)
            out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev) if epi == 2 else None
            for _ in range(20):
                ext().gemm(0, epi, x, w, out, b if epi else None, aux, None, None, False)
            torch.cuda.synchronize()
            tiles = {768: ((M + 127) // 128) * (N // 64), 2304: ((M + 127) // 128) * (N // 192),
                     3072: ((M + 127) // 128) * (N // 128)}[N]
            report(f"{nm} N={N} K={K}", tiles, False)
        # the pruned block's M = 64 GEMMs: split-K slabs (the stamps are the GEMM launch's)
        for (N, K) in ((768, 768), (3072, 768), (768, 3072)):
            x, w = bf(64, K), bf(N, K, scale=0.03)
            out = torch.empty(64, N, dtype=torch.bfloat16, device=dev)
            ws = torch.empty(64 * 64 * N, device=dev)
            for _ in range(20):
                sp, _ = ext().gemm_splitk(0, x, w, out, ws)
            torch.cuda.synchronize()
            report(f"splitk M=64 N={N} K={K} s{sp}", (N // 64) * sp, False)
        print()


if __name__ == "__main__":
    main()
