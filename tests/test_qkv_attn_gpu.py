"""QKV projection + S <= 128 attention forward as ONE launch (csrc/kernels/gemm.hip
gemm_attn_fwd_kernel, ops/kernels.py qkv_attn_fwd) against the two launches it replaces
(linear_fwd + attn_fwd): the projection, the context, lse and the dropout keep bits bit for bit
(packed / padded, with and without dropout, the pruned block's [CLS]-only form with its compact
rows), repeated launches on one exchange epoch with distinct call sites, and a whole training
step of the model with the fusion on / off (FD_FUSE_QKV_ATTN)."""
import pytest
import torch

from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.models import (
    DDoSClassifier, DistilBertConfig)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K

pytestmark = pytest.mark.gpu

H, D = 12, 768


def _problem(B, S, packed, seed, empty=None):
    g = torch.Generator(device="cuda").manual_seed(seed)
    gl = torch.Generator().manual_seed(seed)
    if packed:
        lens = torch.randint(16, S + 1, (B,), generator=gl)
        if empty is not None:
            lens[empty] = 0
        cu = torch.zeros(B + 1, dtype=torch.int32)
        cu[1:] = torch.cumsum(lens, 0)
        rows = (int(cu[-1]) + 127) // 128 * 128 + 64  # + filler rows past cu[B]
        cu = cu.cuda()
        kb = torch.zeros(1, device="cuda")
    else:
        lens = torch.randint(16, S + 1, (B,), generator=gl)
        cu, rows = None, B * S
        mask = (torch.arange(S)[None] < lens[:, None]).cuda()
        kb = K.mask_bias(mask.to(torch.int64))
    x = (torch.randn(rows, D, device="cuda", generator=g)).to(torch.bfloat16)
    w = (torch.randn(3 * D, D, device="cuda", generator=g) * 0.03).to(torch.bfloat16)
    b = torch.randn(3 * D, device="cuda", generator=g) * 0.1
    return x, w, b, kb, cu, lens


def _valid_lse(lse, lens, q_live=0):
    out = []
    for i, n in enumerate(lens.tolist()):
        n = min(n, q_live) if q_live else n
        out.append(lse[i, :, :n].reshape(-1))
    return torch.cat(out)


@pytest.fixture(autouse=True, params=[1, 2])
def mode(request, monkeypatch):
    # 1: tile hand-off, 2: per-(sequence, head) projection into the attention's LDS images
    monkeypatch.setattr(K, "FUSE_QKV_ATTN", request.param)
    return request.param


def _qkv_eq(qkv_f, qkv_r, cu, mode):
    if cu is not None and mode == 2:  # (mode 2: filler rows past cu[B] are zero, never read)
        n = int(cu[-1])
        return torch.equal(qkv_f[:n], qkv_r[:n]) and not qkv_f[n:].any()
    return torch.equal(qkv_f, qkv_r)


@pytest.mark.parametrize("packed", [True, False])
@pytest.mark.parametrize("B,S", [(32, 128), (8, 64), (3, 128)])
def test_fused_qkv_attention_bitwise(packed, B, S, mode):
    x, w, b, kb, cu, lens = _problem(B, S, packed, seed=11 + B + S)
    seed = torch.tensor([9], dtype=torch.int32, device="cuda")
    for p in (0.0, 0.1):
        # (zeroed: rows past a sequence are never written, by either path)
        dm_r, dm_f = [None if d is None else d.zero_() for d in (K.attn_keep_bits(B, S, H, p, "cuda"),
                                                                 K.attn_keep_bits(B, S, H, p, "cuda"))]
        qkv_r = K.linear_fwd(x, w, b)
        ctx_r, lse_r = K.attn_fwd(qkv_r, kb, B, S, H, seed, 21, p, cu, dm_r)
        K.ln_epoch_advance(x.device)
        qkv_f, ctx_f, lse_f = K.qkv_attn_fwd(x, w, b, kb, B, S, H, seed, 21, p, cu, dm_f, xsite=4)
        torch.cuda.synchronize()
        assert _qkv_eq(qkv_f, qkv_r, cu, mode)
        if packed:
            assert torch.equal(ctx_f, ctx_r)  # (the filler rows are zeroed by both)
        else:
            valid = (torch.arange(S)[None] < lens[:, None]).reshape(-1).cuda()
            assert torch.equal(ctx_f[valid], ctx_r[valid])
        assert torch.equal(_valid_lse(lse_f, lens), _valid_lse(lse_r, lens))
        if dm_r is not None:
            assert torch.equal(dm_f, dm_r)
    assert not K.ln_error_flag(x.device)


def test_fused_qkv_attention_repeated_sites(mode):
    """Several fused launches in ONE exchange epoch (distinct call sites, as the layers of one
    forward) and across epochs: each sees only its own tiles' hand-off granules."""
    B, S = 32, 128
    x, w, b, kb, cu, lens = _problem(B, S, True, seed=5)
    seed = torch.tensor([2], dtype=torch.int32, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(8)
    K.ln_epoch_advance(x.device)
    for it in range(6):
        if it == 3:
            K.ln_epoch_advance(x.device)
        xi = (x.float() + torch.randn(x.shape, device="cuda", generator=g)).to(torch.bfloat16)
        qkv_f, ctx_f, _ = K.qkv_attn_fwd(xi, w, b, kb, B, S, H, seed, 30, 0.1, cu, None, xsite=2 * (it % 3))
        qkv_r = K.linear_fwd(xi, w, b)
        ctx_r, _ = K.attn_fwd(qkv_r, kb, B, S, H, seed, 30, 0.1, cu)
        torch.cuda.synchronize()
        assert _qkv_eq(qkv_f, qkv_r, cu, mode) and torch.equal(ctx_f, ctx_r), it
    assert not K.ln_error_flag(x.device)


@pytest.mark.parametrize("packed,empty", [(True, None), (True, 5), (False, None)])
def test_fused_qkv_attention_cls_rows(packed, empty, mode):
    """The pruned block's form: [CLS] query rows only (q_live 1) and the compact [CLS] rows of
    ctx and of the residual stream, bitwise the two-launch path."""
    B, S, Bp = 20, 128, 64
    x, w, b, kb, cu, lens = _problem(B, S, packed, seed=17, empty=empty)
    seed = torch.tensor([4], dtype=torch.int32, device="cuda")
    for p in (0.0, 0.1):
        # (zeroed: rows past a sequence are never written, by either path)
        dm_r, dm_f = [None if d is None else d.zero_() for d in (K.attn_keep_bits(B, S, H, p, "cuda"),
                                                                 K.attn_keep_bits(B, S, H, p, "cuda"))]
        qkv_r = K.linear_fwd(x, w, b)
        ctx_r, lse_r, cxc_r, xc_r = K.attn_fwd(qkv_r, kb, B, S, H, seed, 7, p, cu, dm_r, q_live=1, cls=(x, Bp))
        K.ln_epoch_advance(x.device)
        qkv_f, ctx_f, lse_f, cxc_f, xc_f = K.qkv_attn_fwd(x, w, b, kb, B, S, H, seed, 7, p, cu, dm_f, q_live=1,
                                                          cls=(x, Bp), xsite=10)
        torch.cuda.synchronize()
        assert _qkv_eq(qkv_f, qkv_r, cu, mode)
        assert torch.equal(cxc_f, cxc_r) and torch.equal(xc_f, xc_r)
        assert torch.equal(_valid_lse(lse_f, lens, 1), _valid_lse(lse_r, lens, 1))


def _batch(B, S, seed):
    gen = torch.Generator().manual_seed(seed)
    ids = torch.randint(1000, 2000, (B, S), generator=gen)
    lens = torch.randint(60, 85, (B,), generator=gen)
    mask = (torch.arange(S)[None] < lens[:, None]).long()
    ids = ids * mask
    ids[:, 0] = 101
    labels = torch.randint(0, 2, (B,), generator=gen)
    return ids.cuda(), mask.cuda(), labels.cuda(), int(lens.sum())


@pytest.mark.parametrize("packed,prune", [(True, True), (True, False), (False, True)])
def test_model_step_fused_qkv_attention_bitwise(packed, prune, mode, monkeypatch):
    """A training forward + backward with the fused QKV + attention launches equals the one with
    the separate launches bit for bit (loss, logits, every gradient)."""
    outs = []
    for on in (mode, 0):
        monkeypatch.setattr(K, "FUSE_QKV_ATTN", on)
        m = DDoSClassifier(config=DistilBertConfig(n_layers=3), device="cuda", impl="hip", seed=29)
        m.prune_last = prune
        m.train()
        ids, mask, labels, tokens = _batch(32, 128, seed=77)
        m.zero_grad()
        m.rng.fill_(3)
        loss, logits = m.forward_loss(ids, mask, labels, tokens=tokens if packed else None)
        loss.backward()
        torch.cuda.synchronize()
        outs.append((loss.detach().clone(), logits.detach().clone(), m.arena.grad.clone()))
    (l0, z0, g0), (l1, z1, g1) = outs
    assert torch.equal(z0, z1) and l0.item() == l1.item() and torch.equal(g0, g1)
    K.check_ln_error(ids.device)


@pytest.mark.parametrize("packed,empty", [(True, None), (True, 2), (False, None)])
@pytest.mark.parametrize("B,S", [(32, 128), (8, 64), (5, 128)])
def test_attention_backward_with_projection_bitwise(packed, empty, B, S, mode):
    """attn_bwd_proj (the out-projection's dX computed per (sequence, head) inside the attention
    backward, csrc/kernels/gemm.hip attn_bwd_proj_kernel) == linear_dx + attn_bwd, bit for bit,
    with and without dropout keep bits."""
    if mode != 1:
        pytest.skip("(independent of the forward fusion mode)")
    x, w, b, kb, cu, lens = _problem(B, S, packed, seed=31 + B + S, empty=empty)
    g = torch.Generator(device="cuda").manual_seed(B + S)
    seed = torch.tensor([6], dtype=torch.int32, device="cuda")
    wo = (torch.randn(D, D, device="cuda", generator=g) * 0.03).to(torch.bfloat16)
    dy = (torch.randn(x.shape[0], D, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
    for p in (0.0, 0.1):
        dm = K.attn_keep_bits(B, S, H, p, "cuda")
        if dm is not None:
            dm.zero_()
        qkv = K.linear_fwd(x, w, b)
        ctx, lse = K.attn_fwd(qkv, kb, B, S, H, seed, 12, p, cu, dm)
        ref = K.attn_bwd(qkv, kb, ctx, lse, K.linear_dx(dy, wo), B, S, H, seed, 12, p, cu, dm)
        got = K.attn_bwd_proj(qkv, kb, ctx, lse, dy, wo, B, S, H, seed, 12, p, cu, dm)
        torch.cuda.synchronize()
        if packed:
            assert torch.equal(got, ref)
        else:
            valid = (torch.arange(S)[None] < lens[:, None]).reshape(-1).cuda()
            assert torch.equal(got[valid], ref[valid])


@pytest.mark.parametrize("packed,prune", [(True, True), (False, False)])
def test_model_step_fused_attention_backward_bitwise(packed, prune, mode, monkeypatch):
    """A training step with the out-projection dX inside the attention backward equals the
    two-launch step bit for bit (loss, logits, every gradient)."""
    if mode != 2:
        pytest.skip("(run once, with the default forward)")
    outs = []
    for on in (1, 0):
        monkeypatch.setattr(K, "FUSE_ATTN_BWD", on)
        m = DDoSClassifier(config=DistilBertConfig(n_layers=3), device="cuda", impl="hip", seed=33)
        m.prune_last = prune
        m.train()
        ids, mask, labels, tokens = _batch(32, 128, seed=78)
        m.zero_grad()
        m.rng.fill_(4)
        loss, logits = m.forward_loss(ids, mask, labels, tokens=tokens if packed else None)
        loss.backward()
        torch.cuda.synchronize()
        outs.append((loss.detach().clone(), logits.detach().clone(), m.arena.grad.clone()))
    (l0, z0, g0), (l1, z1, g1) = outs
    assert torch.equal(z0, z1) and l0.item() == l1.item() and torch.equal(g0, g1)


@pytest.mark.parametrize("packed,empty", [(True, None), (True, 5), (False, None)])
def test_compact_attention_backward_with_projection_bitwise(packed, empty, mode):
    """The pruned block's form: the [CLS] rows' out-projection dX (an M = 64 split-K product in the
    two-launch path: 6 partial chains summed in split order) inside the q_live = 1 attention
    backward, which also scatters the residual gradient -- bitwise linear_dx + attn_bwd(dresc=)."""
    if mode != 1:
        pytest.skip("(independent of the forward fusion mode)")
    B, S, Bp = 20, 128, 64
    x, w, b, kb, cu, lens = _problem(B, S, packed, seed=23, empty=empty)
    g = torch.Generator(device="cuda").manual_seed(9)
    seed = torch.tensor([8], dtype=torch.int32, device="cuda")
    wo = (torch.randn(D, D, device="cuda", generator=g) * 0.03).to(torch.bfloat16)
    dyc = (torch.randn(Bp, D, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
    assert K._dx_splits(Bp, D, D) > 1  # (the split-K order is what is being reproduced)
    for p in (0.0, 0.1):
        dm = K.attn_keep_bits(B, S, H, p, "cuda")
        if dm is not None:
            dm.zero_()
        qkv = K.linear_fwd(x, w, b)
        ctx, lse, cxc, xc = K.attn_fwd(qkv, kb, B, S, H, seed, 14, p, cu, dm, q_live=1, cls=(x, Bp))
        ref_q, ref_r = K.attn_bwd(qkv, kb, ctx, lse, K.linear_dx(dyc, wo), B, S, H, seed, 14, p, cu, dm, q_live=1,
                                  dresc=dyc)
        got_q, got_r = K.attn_bwd_proj(qkv, kb, ctx, lse, dyc, wo, B, S, H, seed, 14, p, cu, dm, dresc=dyc)
        torch.cuda.synchronize()
        assert torch.equal(got_r, ref_r)
        assert torch.equal(got_q, ref_q)
