"""LayerNorm fused into the N = 768 GEMMs (csrc/kernels/gemm.hip gemm_ln_kernel).

Forward: y = LN(dropout(x W^T + b) + res) in the GEMM's epilogue (out_lin + sa_layer_norm,
lin2 + output_layer_norm; reference op [ext] modeling_distilbert.py via client1.py:61).
Backward: dy = a Wt^T + res, then the LayerNorm backward from the saved pre-LN sum z, in the
dX GEMM's epilogue.  Checked against a plain fp32 PyTorch reference of the same op and against
the unfused kernels (same counter-hash dropout masks); the cross-tile row-statistic exchange
is checked for timeouts (error flag) and for re-armed counters after many launches and graph
replays.
"""
import pytest
import torch
import torch.nn.functional as F

from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.models import (
    DDoSClassifier, DistilBertConfig)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as kn
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import reference as R

pytestmark = pytest.mark.gpu
DEV = "cuda"
D = 768


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def bf(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).to(DEV)


def seed_t(v=7):
    return torch.tensor([v], dtype=torch.int32, device=DEV)


def affine(seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return ((torch.randn(D, generator=g) * 0.2 + 1).to(DEV), (torch.randn(D, generator=g) * 0.1).to(DEV))


def state_clean(M):
    """No exchange timed out and the epoch advanced (standalone launches start their own)."""
    stats, cnt, err = kn._ln_state(torch.device(DEV), M, D)
    torch.cuda.synchronize()
    return int(err.item()) == 0 and int(cnt[0].item()) > 0


@pytest.fixture(params=[-1, 0, 18])
def ln_cfg(request, monkeypatch):
    """Every instantiated LayerNorm-fused tile configuration (gemm.hip fd_gemm_ln): the default
    (cfg 24, 6-slot ring with the LDS-DMA'd epilogue operands) and the 4- / 8-wave 3-slot rings."""
    monkeypatch.setattr(kn, "LN_CFG", request.param)
    return request.param


@pytest.mark.parametrize("M,K,p", [(2688, 768, 0.0), (2600, 3072, 0.1), (300, 3072, 0.1), (2000, 768, 0.0),
                                   (64, 768, 0.1), (640, 128, 0.0)])
def test_linear_ln_fwd(M, K, p, ln_cfg):
    x, w, res = bf(M, K, seed=1), bf(D, K, scale=0.03, seed=2), bf(M, D, seed=3)
    b = (torch.randn(D, generator=torch.Generator().manual_seed(4)) * 0.1).to(DEV)
    gamma, beta = affine(5)
    y, z, mean, rstd = kn.linear_ln_fwd(x, w, b, res, gamma, beta, 1e-12, seed_t(9), 33, p)
    f = x.float() @ w.float().t() + b
    zr = R.dropout_ref(f, p, 9, 33) + res.float()
    assert rel_err(z, zr) < 1e-2
    yr = F.layer_norm(zr, (D,), gamma, beta, 1e-12)
    assert rel_err(y, yr) < 1e-2
    # the statistics are those of the stored (bf16) pre-LN sum
    zf = z.float()
    assert torch.allclose(mean, zf.mean(1), atol=1e-4, rtol=1e-4)
    assert torch.allclose(rstd, torch.rsqrt(zf.var(1, unbiased=False) + 1e-12), rtol=1e-3)
    # the unfused kernels draw the same dropout masks
    y2, _, _ = kn.ln_fwd(kn.linear_fwd(x, w, b), res, gamma, beta, 1e-12, seed_t(9), 33, p)
    assert rel_err(y, y2) < 2e-2
    assert state_clean(M)


def test_fused_grid_limited_to_one_resident_round(monkeypatch):
    """Row blocks wait on each other's statistics, so the fused grid must fit one round of the
    CUs: 21 row blocks x 12 column tiles of 128 x 64 at N = 768, or -- with the two-K-half
    kernels -- 21 row blocks of 256-row tiles.  A larger M is refused by the launcher and the model
    takes the separate LayerNorm kernels (ln_fusable)."""
    M, K = 6000, 768
    x, w, res = bf(M, K, seed=1), bf(D, K, scale=0.03, seed=2), bf(M, D, seed=3)
    gamma, beta = affine(5)
    monkeypatch.setattr(kn, "LN2", False)
    assert kn.ln_fusable(2688, D) and not kn.ln_fusable(2689, D) and not kn.ln_fusable(4096, D)
    with pytest.raises(RuntimeError):
        kn.linear_ln_fwd(x[:4096], w, torch.zeros(D, device=DEV), res[:4096], gamma, beta, 1e-12, seed_t(9), 33, 0.0)
    monkeypatch.setattr(kn, "LN2", True)
    assert kn.ln_fusable(4096, D) and kn.ln_fusable(5376, D) and not kn.ln_fusable(5377, D)
    with pytest.raises(RuntimeError):
        kn.linear_ln_fwd(x, w, torch.zeros(D, device=DEV), res, gamma, beta, 1e-12, seed_t(9), 33, 0.0)


@pytest.mark.parametrize("M,K,p", [(5000, 3072, 0.1), (5000, 768, 0.0), (4000, 2304, 0.1)])
def test_256_row_two_k_half_tiles(M, K, p):
    """Past one round of 128-row tiles (the seq256 bs64 distillation batch: ~5.1 k packed rows) the
    fused kernels run 256-row two-K-half tiles: forward and backward (both B layouts) against fp32
    references and the unfused kernels."""
    x, w, res = bf(M, K, seed=41), bf(D, K, scale=0.03, seed=42), bf(M, D, seed=43)
    b = (torch.randn(D, generator=torch.Generator().manual_seed(44)) * 0.1).to(DEV)
    gamma, beta = affine(45)
    y, z, mean, rstd = kn.linear_ln_fwd(x, w, b, res, gamma, beta, 1e-12, seed_t(9), 33, p)
    zr = R.dropout_ref(x.float() @ w.float().t() + b, p, 9, 33) + res.float()
    assert rel_err(z, zr) < 1e-2
    assert rel_err(y, F.layer_norm(zr, (D,), gamma, beta, 1e-12)) < 1e-2
    y2, _, _ = kn.ln_fwd(kn.linear_fwd(x, w, b), res, gamma, beta, 1e-12, seed_t(9), 33, p)
    assert rel_err(y, y2) < 2e-2
    a = bf(M, K, scale=0.5, seed=46)
    for b_mn in (False, True):
        wt = bf(K, D, scale=0.03, seed=47) if b_mn else bf(D, K, scale=0.03, seed=47)
        dgamma, dbeta, dbias = (torch.zeros(D, device=DEV) for _ in range(3))
        dz, dx = kn.linear_dx_ln_bwd(a, wt, res, z, gamma, mean, rstd, dgamma, dbeta, dbias, seed_t(9), 33, p,
                                     b_mn=b_mn)
        dy = a.float() @ (wt.float() if b_mn else wt.float().t()) + res.float()
        zf = z.float().requires_grad_(True)
        gf, bf_ = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
        gz, gg, gb = torch.autograd.grad(F.layer_norm(zf, (D,), gf, bf_, 1e-12), [zf, gf, bf_], dy)
        assert rel_err(dz, gz) < 2e-2
        assert rel_err(dx, R.dropout_ref(gz, p, 9, 33)) < 2e-2
        assert rel_err(dgamma, gg) < 1e-2 and rel_err(dbeta, gb) < 1e-2
    assert state_clean(M)


def test_linear_ln_fwd_packed_row_map():
    """Packed rows hash their dropout by the padded row (row_map), like ln_fwd."""
    M, K, p = 1000, 3072, 0.1
    x, w, res = bf(M, K, seed=11), bf(D, K, scale=0.03, seed=12), bf(M, D, seed=13)
    b = torch.zeros(D, device=DEV)
    gamma, beta = affine(14)
    row_map = (torch.arange(M, dtype=torch.int32, device=DEV) * 3 + 1)
    row_map[-5:] = -1  # bucket filler rows
    y, z, _, _ = kn.linear_ln_fwd(x, w, b, res, gamma, beta, 1e-12, seed_t(5), 17, p, row_map)
    y2, _, _ = kn.ln_fwd(kn.linear_fwd(x, w, b), res, gamma, beta, 1e-12, seed_t(5), 17, p, row_map)
    assert rel_err(y, y2) < 2e-2
    # ~p of the entries are dropped: there z is exactly the residual
    dropped = (z.float() - res.float()).abs() == 0
    assert 0.07 < dropped.float().mean().item() < 0.13


@pytest.mark.parametrize("M,K,p,defer", [(2688, 3072, 0.0, False), (2600, 2304, 0.1, True), (300, 2304, 0.1, False),
                                         (130, 3072, 0.0, True), (700, 128, 0.1, False)])
def test_linear_dx_ln_bwd(M, K, p, defer, ln_cfg):
    gamma, beta = affine(21)
    x2, w2, r2 = bf(M, D, seed=22), bf(D, D, scale=0.03, seed=23), bf(M, D, seed=24)
    b2 = torch.zeros(D, device=DEV)
    _, z, mean, rstd = kn.linear_ln_fwd(x2, w2, b2, r2, gamma, beta, 1e-12, seed_t(9), 33, p)
    a, wt, res = bf(M, K, scale=0.5, seed=25), bf(D, K, scale=0.03, seed=26), bf(M, D, scale=0.5, seed=27)
    dgamma, dbeta, dbias = (torch.full((D,), 3.0, device=DEV) for _ in range(3))
    jobs = [] if defer else None
    dz, dx = kn.linear_dx_ln_bwd(a, wt, res, z, gamma, mean, rstd, dgamma, dbeta, dbias, seed_t(9), 33, p,
                                 accumulate=False, jobs=jobs)
    if defer:
        assert len(jobs) == 1
        kn.colsum_flush(jobs)
    # fp32 reference: LayerNorm backward of y = LN(z) with dy = a wt^T + res
    dy = a.float() @ wt.float().t() + res.float()
    zf = z.float().requires_grad_(True)
    gf, bf_ = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    yr = F.layer_norm(zf, (D,), gf, bf_, 1e-12)
    gz, gg, gb = torch.autograd.grad(yr, [zf, gf, bf_], dy)
    assert rel_err(dz, gz) < 2e-2
    dx_ref = R.dropout_ref(gz, p, 9, 33)
    assert rel_err(dx, dx_ref) < 2e-2
    assert rel_err(dgamma, gg) < 1e-2
    assert rel_err(dbeta, gb) < 1e-2
    assert rel_err(dbias, dx_ref.sum(0)) < 1e-2
    # unfused: dX GEMM (+ residual), then the LN backward from z
    dh = kn.linear_dx(a, wt.t().contiguous(), res=res)
    e1, e2, e3 = (torch.empty(D, device=DEV) for _ in range(3))
    dz2, dx2 = kn.ln_bwd(dh, z, None, gamma, mean, rstd, e1, e2, e3, seed_t(9), 33, p, zin=True)
    assert rel_err(dz, dz2) < 2e-2 and rel_err(dx, dx2) < 2e-2
    assert rel_err(dgamma, e1) < 2e-2 and rel_err(dbeta, e2) < 2e-2 and rel_err(dbias, e3) < 2e-2
    # accumulate adds onto the existing gradient
    acc = [t.clone() for t in (dgamma, dbeta, dbias)]
    kn.linear_dx_ln_bwd(a, wt, res, z, gamma, mean, rstd, dgamma, dbeta, dbias, seed_t(9), 33, p, accumulate=True)
    for t, t0 in zip((dgamma, dbeta, dbias), acc):
        assert torch.allclose(t, 2 * t0, rtol=1e-5, atol=1e-5)
    assert state_clean(M)


@pytest.mark.parametrize("bwd,b_mn", [(False, False), (True, False), (True, True)])
def test_two_k_half_tiles_match_one_pass(bwd, b_mn, monkeypatch):
    """K >= FD_GEMM_LN2_MINK: two blocks per 128 x 128 product tile run half the K loop each and
    trade fp32 column-half partials through write-through stores and a tagged flag
    (gemm.hip gemm_ln2_kernel).  Equal to the one-pass kernel up to fp32 summation order,
    bitwise repeatable (the pair's sum commutes), no exchange timeout."""
    M, K, p = 2600, 3072, 0.1
    gamma, beta = affine(31)
    b = (torch.randn(D, generator=torch.Generator().manual_seed(32)) * 0.1).to(DEV)
    res = bf(M, D, seed=33)
    if not bwd:
        x, w = bf(M, K, seed=34), bf(D, K, scale=0.03, seed=35)
        run = lambda: kn.linear_ln_fwd(x, w, b, res, gamma, beta, 1e-12, seed_t(9), 33, p)[:2]
    else:
        x2, w2 = bf(M, D, seed=36), bf(D, D, scale=0.03, seed=37)
        _, z, mean, rstd = kn.linear_ln_fwd(x2, w2, b, res, gamma, beta, 1e-12, seed_t(9), 33, p)
        a = bf(M, K, scale=0.5, seed=38)
        wt = bf(K, D, scale=0.03, seed=39) if b_mn else bf(D, K, scale=0.03, seed=39)
        sinks = [torch.zeros(D, device=DEV) for _ in range(3)]
        run = lambda: kn.linear_dx_ln_bwd(a, wt, res, z, gamma, mean, rstd, *sinks, seed_t(9), 33, p,
                                          b_mn=b_mn) + (sinks[0].clone(),)
    monkeypatch.setattr(kn, "LN2", True)
    r1 = [t.clone() for t in run()]
    r2 = [t.clone() for t in run()]
    monkeypatch.setattr(kn, "LN2", False)
    r0 = [t.clone() for t in run()]
    torch.cuda.synchronize()
    for t1, t2, t0 in zip(r1, r2, r0):
        assert torch.equal(t1, t2)
        assert rel_err(t1, t0) < 2e-2
    assert state_clean(M)


def test_many_launches_and_graph_replay_rearm_counters():
    """Standalone launches start a fresh exchange epoch each (graph replays re-run the advance);
    results are bitwise reproducible across launches (fixed-order merge)."""
    M, K = 2688, 3072
    x, w, res = bf(M, K, seed=31), bf(D, K, scale=0.03, seed=32), bf(M, D, seed=33)
    b = torch.zeros(D, device=DEV)
    gamma, beta = affine(34)
    y0, z0, m0, r0 = kn.linear_ln_fwd(x, w, b, res, gamma, beta, 1e-12, seed_t(3), 7, 0.1)
    dg, db, dbi = (torch.empty(D, device=DEV) for _ in range(3))
    for _ in range(100):
        y, z, m, r = kn.linear_ln_fwd(x, w, b, res, gamma, beta, 1e-12, seed_t(3), 7, 0.1)
        dz, dx = kn.linear_dx_ln_bwd(x, w, res, z0, gamma, m0, r0, dg, db, dbi, seed_t(3), 7, 0.1)
    torch.cuda.synchronize()
    assert torch.equal(y, y0) and torch.equal(z, z0) and torch.equal(m, m0) and torch.equal(r, r0)
    assert state_clean(M)
    out = torch.empty_like(y0)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        kn.linear_ln_fwd(x, w, b, res, gamma, beta, 1e-12, seed_t(3), 7, 0.1)
    torch.cuda.current_stream().wait_stream(s)
    sd = seed_t(3)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        yg, _, _, _ = kn.linear_ln_fwd(x, w, b, res, gamma, beta, 1e-12, sd, 7, 0.1)
        out.copy_(yg)
    for _ in range(5):
        out.zero_()
        gr.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, y0)
    assert state_clean(M)


def _grads(fuse, packed, seed=21):
    cfg = DistilBertConfig(n_layers=3)
    m = DDoSClassifier(config=cfg, device=DEV, impl="hip", seed=seed)
    m.fuse_ln = fuse
    m.train()
    g = torch.Generator().manual_seed(0)
    B, S = 16, 128
    ids = torch.randint(1000, 2000, (B, S), generator=g)
    lens = torch.randint(S // 3, S + 1, (B,), generator=g)
    mask = (torch.arange(S)[None] < lens[:, None]).long()
    ids = (ids * mask).to(DEV)
    ids[:, 0] = 101
    labels = torch.randint(0, 2, (B,), generator=g).to(DEV)
    m.rng.zero_()
    m.zero_grad()
    loss, logits = m.forward_loss(ids, mask.to(DEV), labels, tokens=int(lens.sum()) if packed else None)
    loss.backward()
    torch.cuda.synchronize()
    return m, loss.item(), logits.float()


@pytest.mark.parametrize("packed", [False, True])
def test_model_fused_ln_matches_unfused(packed):
    """Whole model (3 blocks, dropout on, identical masks): fused-LN gradients vs the unfused
    kernels, per tensor ||a - b|| / ||b|| (the two differ only in bf16 rounding points)."""
    mf, lf, zf = _grads(True, packed)
    mu, lu, zu = _grads(False, packed)
    assert abs(lf - lu) < 1e-2 * max(1.0, abs(lu))
    assert rel_err(zf, zu) < 2e-2
    worst = ("", 0.0)
    for name in mu.state_dict().keys():
        if name.endswith("k_lin.bias"):
            continue
        a, b = mf.dense_grad(name).float(), mu.dense_grad(name).float()
        e = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
        worst = max(worst, (name, e), key=lambda t: t[1])
    assert worst[1] < 2e-2, worst
    assert kn.ln_error_flag(DEV) == 0


def test_explicit_call_sites_share_one_epoch():
    """Launches that pass their exchange call site (``ln_xsite``, as the model does) run in ONE
    epoch -- advanced once, like the model's embedding launch does -- and give the same results
    as standalone launches."""
    M, K = 2688, 768
    x, w, res = bf(M, K, seed=41), bf(D, K, scale=0.03, seed=42), bf(M, D, seed=43)
    b = torch.zeros(D, device=DEV)
    gamma, beta = affine(44)
    y0, z0, m0, r0 = kn.linear_ln_fwd(x, w, b, res, gamma, beta, 1e-12, seed_t(3), 7, 0.1)
    dg, db, dbi = (torch.empty(D, device=DEV) for _ in range(3))
    dz0, _ = kn.linear_dx_ln_bwd(x, w, res, z0, gamma, m0, r0, dg, db, dbi, seed_t(3), 7, 0.1)
    for _ in range(3):
        kn.ln_epoch_advance(DEV)
        outs = []
        for layer in range(6):
            y, z, m, r = kn.linear_ln_fwd(x, w, b, res, gamma, beta, 1e-12, seed_t(3), 7, 0.1,
                                          xsite=kn.ln_xsite(layer, layer % 2, False))
            dz, _ = kn.linear_dx_ln_bwd(x, w, res, z0, gamma, m0, r0, dg, db, dbi, seed_t(3), 7, 0.1,
                                        xsite=kn.ln_xsite(layer, layer % 2, True))
            outs.append((y, dz))
        torch.cuda.synchronize()
        for y, dz in outs:
            assert torch.equal(y, y0) and torch.equal(dz, dz0)
    assert state_clean(M)


def test_rendezvous_timeout_is_detected_and_fatal():
    """a timed-out row-block rendezvous (forced with diag 64: a tag no launch writes)
    sets the error flag, and the host check raises instead of training on wrong statistics."""
    M, K = 256, 768  # 2 row blocks x 12 tiles, each waits the 0.25 s bound once
    x, w, res = bf(M, K, seed=51), bf(D, K, scale=0.03, seed=52), bf(M, D, seed=53)
    gamma, beta = affine(54)
    _, _, err = kn._ln_state(torch.device(DEV), M, D)
    err.zero_()
    kn.check_ln_error(DEV)
    try:
        kn.ln_set_diag(64)
        kn.linear_ln_fwd(x, w, torch.zeros(D, device=DEV), res, gamma, beta, 1e-12, seed_t(3), 7, 0.0)
        torch.cuda.synchronize()
    finally:
        kn.ln_set_diag(0)
    assert kn.ln_error_flag(DEV) != 0
    with pytest.raises(RuntimeError, match="timed out"):
        kn.check_ln_error(DEV)
    err.zero_()
    kn.linear_ln_fwd(x, w, torch.zeros(D, device=DEV), res, gamma, beta, 1e-12, seed_t(3), 7, 0.0)
    torch.cuda.synchronize()
    kn.check_ln_error(DEV)


def test_granule_tags_wrap_clears_stats():
    """a granule tag is (epoch * 128 + site + 1) mod 2^32, so tags repeat every 2^25
    epochs.  The epoch launch (emb_fwd) zeroes every granule when the epoch crosses such a
    multiple -- a row block's statistics untouched since then can never pass for fresh ones --
    and the fused LayerNorm still matches the unfused kernels right after the wrap."""
    dev = torch.device(DEV)
    M, K = 2688, 768
    stats, cnt, err = kn._ln_state(dev, M, D)
    T, S = 256, 128
    ids = torch.randint(0, 1000, (T,), device=DEV)
    word, pos = bf(1000, D, seed=11), bf(512, D, seed=12)
    gamma, beta = affine(13)
    # one epoch short of a multiple of 2^25: the next epoch launch must not clear anything
    cnt[0] = (1 << 25) - 2
    stats.fill_(0x1234567800000000)
    kn.emb_fwd(ids, word, pos, gamma, beta, S, 1e-12, seed_t(1), 1, 0.0, ln_epoch=cnt, ln_stats=stats)
    torch.cuda.synchronize()
    assert int(cnt[0].item()) == (1 << 25) - 1 and bool((stats == 0x1234567800000000).all())
    kn.emb_fwd(ids, word, pos, gamma, beta, S, 1e-12, seed_t(1), 1, 0.0, ln_epoch=cnt, ln_stats=stats)
    torch.cuda.synchronize()
    assert int(cnt[0].item()) == 1 << 25 and int(stats.count_nonzero().item()) == 0
    # the exchange works at the wrapped epoch (tags 1..128 again)
    x, w, res = bf(M, K, seed=1), bf(D, K, scale=0.03, seed=2), bf(M, D, seed=3)
    b = (torch.randn(D, generator=torch.Generator().manual_seed(4)) * 0.1).to(DEV)
    y, _, _, _ = kn.linear_ln_fwd(x, w, b, res, gamma, beta, 1e-12, seed_t(9), 33, 0.0, xsite=5)
    y2, _, _ = kn.ln_fwd(kn.linear_fwd(x, w, b), res, gamma, beta, 1e-12, seed_t(9), 33, 0.0)
    assert rel_err(y, y2) < 2e-2
    assert int(err.item()) == 0


def test_gemm_override_rejects_uninstantiated_cfg():
    """a tuning override naming a configuration that is not compiled in is refused
    (fd_gemm_set_cfg) instead of making later launches fail."""
    from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops._ext import ext
    with pytest.raises(RuntimeError):
        ext().gemm_set_cfg(0, 2, -1)   # cfg 2 was measured and removed
    ext().gemm_set_cfg(0, 8, -1)       # an instantiated one is accepted
    x, w = bf(256, 768, seed=1), bf(768, 768, scale=0.03, seed=2)
    y = kn.linear_fwd(x, w, None)
    ext().gemm_set_cfg(0, -1, -1)
    assert rel_err(y, x.float() @ w.float().t()) < 1e-2
