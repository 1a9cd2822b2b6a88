"""Split-K small-M GEMMs (csrc/kernels/splitk.hip + gemm.hip fd_gemm_f32_splits): the pruned
last block's M = 64 [CLS]-row GEMMs run as fp32 slabs over K + one reduce/epilogue launch.  Every
epilogue is checked against a plain fp32 torch reference of the same op, and the LayerNorm ones
against the one-pass LayerNorm-fused GEMM (same math, fp32 summation order aside)."""
import pytest
import torch

from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import dropout as DR
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops._ext import ext

pytestmark = pytest.mark.gpu
DEV = "cuda"
D = 768


def bf(*s, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*s, generator=g) * scale).to(torch.bfloat16).to(DEV)


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()


@pytest.fixture
def no_splitk(monkeypatch):
    monkeypatch.setattr(K, "SPLITK_MAX_M", 0)


@pytest.mark.parametrize("M,N,K_", [(64, 768, 768), (64, 3072, 768), (64, 768, 3072), (40, 768, 2304), (1, 64, 64)])
def test_splitk_plain_and_bias(M, N, K_):
    x, w = bf(M, K_, seed=1), bf(N, K_, scale=0.05, seed=2)
    b = torch.randn(N, device=DEV) * 0.1
    ref = x.float() @ w.float().t()
    y = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ws = torch.full((64 * M * N,), float("nan"), device=DEV)
    splits, _ = ext().gemm_splitk(0, x, w, y, ws)
    assert splits >= 1 and (K_ // 64) % splits == 0
    assert rel(y, ref) < 5e-3
    splits, _ = ext().gemm_splitk(1, x, w, y, ws, bias=b)
    assert rel(y, ref + b) < 5e-3
    # explicit split counts agree with each other to fp32 order
    for s in (1, 2):
        if (K_ // 64) % s:
            continue
        ext().gemm_splitk(1, x, w, y, ws, splits=s, bias=b)
        assert rel(y, ref + b) < 5e-3


def test_splitk_dispatch_covers_linear_wrappers():
    """linear_fwd / linear_dx route M <= 64 through the split-K path (and give the same result
    as the one-pass kernels up to rounding)."""
    M, N, K_ = 64, 3072, 768
    x, w = bf(M, K_, seed=3), bf(N, K_, scale=0.05, seed=4)
    b = torch.randn(N, device=DEV) * 0.1
    g, u = K.linear_fwd(x, w, b, gelu=True)
    ref = x.float() @ w.float().t() + b
    assert rel(u, ref) < 5e-3
    assert rel(g, torch.nn.functional.gelu(u.float())) < 5e-3
    # GELU' with the re-created activation and the fused bias-gradient column partials
    dy = bf(M, N, seed=5)
    wt2 = bf(D, N, scale=0.03, seed=6)          # lin2 weight [768, 3072] -> dx = dy @ W2
    uu = bf(M, N, seed=7)
    jobs, out = [], torch.zeros(N, device=DEV)
    g_out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    du = K.linear_dx(bf(M, D, seed=8), wt2, gelu_u=uu, colsum=(jobs, out, False), aux_out=g_out)
    K.colsum_flush(jobs)
    torch.cuda.synchronize()
    a8 = bf(M, D, seed=8).float()
    uf = uu.float().requires_grad_(True)
    gref = torch.autograd.grad(torch.nn.functional.gelu(uf), uf, a8 @ wt2.float())[0]
    assert rel(du, gref) < 1e-2
    assert torch.equal(g_out, torch.nn.functional.gelu(uu.float()).to(torch.bfloat16)) or \
        rel(g_out, torch.nn.functional.gelu(uu.float())) < 5e-3
    assert rel(out, du.float().sum(0)) < 1e-5  # sums of the stored bf16 values
    # residual epilogue
    res = bf(M, D, seed=9)
    dx = K.linear_dx(dy, wt2.t().contiguous(), res=res)
    assert rel(dx, dy.float() @ wt2.float().t() + res.float()) < 5e-3


@pytest.mark.parametrize("p,rowmap", [(0.0, False), (0.1, False), (0.1, True)])
def test_splitk_ln_forward_matches_fused_and_reference(p, rowmap):
    M, K_ = 64, 3072
    x, w, res = bf(M, K_, seed=11), bf(D, K_, scale=0.03, seed=12), bf(M, D, seed=13)
    b = torch.randn(D, device=DEV) * 0.1
    gamma = 1 + 0.1 * torch.randn(D, device=DEV)
    beta = 0.1 * torch.randn(D, device=DEV)
    seed = torch.tensor([7], dtype=torch.int32, device=DEV)
    rm = (torch.arange(M, device=DEV, dtype=torch.int32) * 128) if rowmap else None
    y, z, mean, rstd = K.linear_ln_fwd(x, w, b, res, gamma, beta, 1e-12, seed, 9, p, rm)
    # fp32 reference of the same op (dropout from the same hash)
    f = x.float() @ w.float().t() + b
    hrow = rm.long() if rm is not None else torch.arange(M, device=DEV)
    if p:
        idx = hrow[:, None] * D + torch.arange(D, device=DEV)[None]
        keep = DR.keep_t(DR.site_seed(int(seed.item()), 9), idx, DR.threshold(p)).float()
    zr = (f * keep / (1 - p) if p else f) + res.float()
    zr_b = zr.to(torch.bfloat16).float()
    yr = torch.nn.functional.layer_norm(zr_b, (D,), gamma, beta, 1e-12)
    assert rel(z, zr) < 5e-3
    assert rel(y, yr) < 1e-2
    assert rel(mean, zr_b.mean(1)) < 1e-3
    # the one-pass LayerNorm-fused GEMM on the same operands
    K.SPLITK_MAX_M, old = 0, K.SPLITK_MAX_M
    try:
        y1, z1, m1, r1 = K.linear_ln_fwd(x, w, b, res, gamma, beta, 1e-12, seed, 9, p, rm)
    finally:
        K.SPLITK_MAX_M = old
    assert rel(y, y1) < 5e-3 and rel(z, z1) < 5e-3 and rel(rstd, r1) < 1e-3


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_splitk_ln_backward_matches_fused(p):
    M, K_ = 64, 3072
    a, wt, res = bf(M, K_, scale=0.5, seed=21), bf(D, K_, scale=0.03, seed=22), bf(M, D, seed=23)
    z = bf(M, D, seed=24)
    gamma = 1 + 0.1 * torch.randn(D, device=DEV)
    zf = z.float()
    mean, rstd = zf.mean(1), torch.rsqrt(zf.var(1, unbiased=False) + 1e-12)
    seed = torch.tensor([3], dtype=torch.int32, device=DEV)
    outs = []
    for lim in (K.SPLITK_MAX_M, 0):
        old, K.SPLITK_MAX_M = K.SPLITK_MAX_M, lim
        try:
            dg, db, dbi = (torch.zeros(D, device=DEV) for _ in range(3))
            dz, dx = K.linear_dx_ln_bwd(a, wt, res, z, gamma, mean, rstd, dg, db, dbi, seed, 17, p)
            torch.cuda.synchronize()
            outs.append((dz.clone(), dx.clone(), dg.clone(), db.clone(), dbi.clone()))
        finally:
            K.SPLITK_MAX_M = old
    # fp32 reference: dy = a wt^T + res; y = LN(z) -> dz; dx = dropout'(dz)
    dy = a.float() @ wt.float().t() + res.float()
    xh = (zf - mean[:, None]) * rstd[:, None]
    gd = gamma * dy
    dzr = rstd[:, None] * (gd - gd.mean(1, keepdim=True) - xh * (gd * xh).mean(1, keepdim=True))
    for (dz, dx, dg, db, dbi) in outs:
        assert rel(dz, dzr) < 1e-2
        assert rel(dg, (dy * xh).sum(0)) < 5e-3
        assert rel(db, dy.sum(0)) < 5e-3
        assert rel(dbi, dx.float().sum(0)) < 1e-2
    for u, v in zip(outs[0], outs[1]):
        assert rel(u, v) < 5e-3


def test_splitk_graph_replay_stable():
    """The slab workspace is shared by every small-M call: a captured sequence of calls replays
    to bitwise the eager results."""
    M = 64
    x, w1, w2 = bf(M, 768, seed=31), bf(3072, 768, scale=0.03, seed=32), bf(768, 3072, scale=0.03, seed=33)
    b1, b2 = torch.zeros(3072, device=DEV), torch.zeros(768, device=DEV)

    def run():
        g, _ = K.linear_fwd(x, w1, b1, gelu=True)
        return K.linear_fwd(g, w2, b2)
    eager = run().clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        run()
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        out = run()
    for _ in range(3):
        out.fill_(0)
        gr.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, eager)
