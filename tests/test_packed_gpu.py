"""Unpadded (packed-token) HIP path == padded path.

Padding positions never reach a real token (keys are masked) or the loss (the
head reads [CLS]), so running the transformer blocks on the real tokens only is
the same math.  The packed path also hashes dropout by the padded row, so even
with dropout on the two paths draw identical masks.
"""
import pytest
import torch

from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.engine import (
    ArenaAdam, GraphedTrainStep, make_step_fn)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.models import (
    DDoSClassifier, DistilBertConfig)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K

pytestmark = pytest.mark.gpu


def _batch(B, S, lo, hi, seed=0):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(1000, 2000, (B, S), generator=g)
    lens = torch.randint(lo, hi + 1, (B,), generator=g)
    mask = (torch.arange(S)[None] < lens[:, None]).long()
    ids = ids * mask
    ids[:, 0] = 101
    labels = torch.randint(0, 2, (B,), generator=g)
    return ids.cuda(), mask.cuda(), labels.cuda(), int(lens.sum())


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-8)).item()


_LENS = {128: [128, 77, 64, 1, 100, 65, 17, 16], 256: [256, 77, 129, 1, 200, 65, 33, 192],
         512: [512, 300, 129, 1, 450, 65, 511, 257]}


@pytest.mark.parametrize("S", [128, 256, 512])  # one-block-per-(b,h) kernels (S <= 128) and the 64-row tiles
def test_varlen_attention_matches_padded(S):
    B, H = 8, 12
    g = torch.Generator(device="cuda").manual_seed(1)
    lens = torch.tensor(_LENS[S])
    qkv_pad = (torch.randn(B * S, 3 * H * 64, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    mask = (torch.arange(S)[None] < lens[:, None]).cuda()
    kb = K.mask_bias(mask.to(torch.int64))
    seed = torch.tensor([7], dtype=torch.int32, device="cuda")
    idx = torch.nonzero(mask.reshape(-1)).squeeze(1)
    cu = torch.zeros(B + 1, dtype=torch.int32, device="cuda")
    cu[1:] = torch.cumsum(lens, 0).to(torch.int32).cuda()
    qkv = torch.cat([qkv_pad.index_select(0, idx), torch.zeros(64, 3 * H * 64, dtype=torch.bfloat16,
                                                                 device="cuda")])  # + filler rows
    # (S > 128: the varlen launch pair's length split off -- the same 64-row kernels as the padded
    # layout, so bitwise; the split itself: test_varlen_split_dispatch below)
    prev = K.ext().attn_set_split(0)
    try:
        for p in (0.0, 0.1):
            ctx_p, lse_p = K.attn_fwd(qkv_pad, kb, B, S, H, seed, 40, p)
            ctx_v, lse_v = K.attn_fwd(qkv, kb, B, S, H, seed, 40, p, cu=cu)
            n = int(cu[-1])
            assert torch.equal(ctx_v[:n], ctx_p.index_select(0, idx))
            assert not ctx_v[n:].any()  # filler rows untouched (zero)
            dctx_pad = (torch.randn(B * S, H * 64, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
            dctx_pad = dctx_pad * mask.reshape(-1, 1)  # padding rows carry no gradient
            dctx = torch.cat([dctx_pad.index_select(0, idx), torch.zeros(64, H * 64, dtype=torch.bfloat16,
                                                                          device="cuda")])
            d_p = K.attn_bwd(qkv_pad, kb, ctx_p, lse_p, dctx_pad, B, S, H, seed, 40, p)
            d_v = K.attn_bwd(qkv, kb, ctx_v, lse_v, dctx, B, S, H, seed, 40, p, cu=cu)
            assert rel(d_v[:n], d_p.index_select(0, idx)) < 1e-6
            assert not d_v[n:].any()
    finally:
        K.ext().attn_set_split(prev)


def _attn_ref(qkv, lens, H, scale=0.125):
    """fp32 attention of each packed sequence (no dropout): ctx rows [n, H 64]."""
    D = H * 64
    out, t0 = [], 0
    for L in lens.tolist():
        x = qkv[t0:t0 + L].float().view(L, 3, H, 64)
        q, k, v = x[:, 0].transpose(0, 1), x[:, 1].transpose(0, 1), x[:, 2].transpose(0, 1)
        pr = torch.softmax(q @ k.transpose(1, 2) * scale, -1)
        out.append((pr @ v).transpose(0, 1).reshape(L, D))
        t0 += L
    return torch.cat(out)


@pytest.mark.parametrize("S", [256, 512])
def test_varlen_split_dispatch(S):
    """Varlen at S > 128 (FD_ATTN_SPLIT, default on): sequences of <= 128 tokens go to the S <= 128
    whole-row kernels, longer ones to the 64-row kernels, in one launch pair.  Against the 64-row
    kernels alone: the long sequences are bitwise theirs; the short ones agree to bf16 rounding
    with the SAME dropout masks (a different mask would differ by O(1)); both match fp32 at p = 0;
    the filler rows stay zero."""
    B, H = 8, 12
    g = torch.Generator(device="cuda").manual_seed(3)
    lens = torch.tensor(_LENS[S])
    n = int(lens.sum())
    cu = torch.zeros(B + 1, dtype=torch.int32, device="cuda")
    cu[1:] = torch.cumsum(lens, 0).to(torch.int32).cuda()
    qkv = torch.cat([(torch.randn(n, 3 * H * 64, device="cuda", generator=g) * 0.5).to(torch.bfloat16),
                     torch.zeros(64, 3 * H * 64, dtype=torch.bfloat16, device="cuda")])
    dctx = torch.cat([(torch.randn(n, H * 64, device="cuda", generator=g) * 0.5).to(torch.bfloat16),
                      torch.zeros(64, H * 64, dtype=torch.bfloat16, device="cuda")])
    kb = K.mask_bias(torch.ones(B, S, dtype=torch.int64, device="cuda"))  # (varlen: not read)
    seed = torch.tensor([11], dtype=torch.int32, device="cuda")
    short = torch.cat([torch.full((L,), L <= 128, dtype=torch.bool) for L in lens.tolist()]).cuda()
    assert short.any() and (~short).any()
    res = {}
    prev = K.ext().attn_set_split(1)
    try:
        for split in (0, 1):
            K.ext().attn_set_split(split)
            for p in (0.0, 0.1):
                ctx, lse = K.attn_fwd(qkv, kb, B, S, H, seed, 41, p, cu=cu)
                d = K.attn_bwd(qkv, kb, ctx, lse, dctx, B, S, H, seed, 41, p, cu=cu)
                torch.cuda.synchronize()
                assert not ctx[n:].any() and not d[n:].any()
                res[split, p] = (ctx[:n].clone(), d[:n].clone())
    finally:
        K.ext().attn_set_split(prev)
    ref = _attn_ref(qkv[:n], lens, H)
    for p in (0.0, 0.1):
        (c0, d0), (c1, d1) = res[0, p], res[1, p]
        assert torch.equal(c1[~short], c0[~short]) and torch.equal(d1[~short], d0[~short])
        assert rel(c1[short], c0[short]) < 1e-2, rel(c1[short], c0[short])
        assert rel(d1[short], d0[short]) < 2e-2, rel(d1[short], d0[short])
    assert rel(res[1, 0.0][0], ref) < 1e-2 and rel(res[0, 0.0][0], ref) < 1e-2


@pytest.mark.parametrize("train", [False, True])
def test_packed_model_matches_padded(train):
    cfg = DistilBertConfig(n_layers=2)
    m = DDoSClassifier(config=cfg, device="cuda", impl="hip", seed=4)
    m.train(train)
    ids, mask, labels, tokens = _batch(16, 128, 70, 90)
    assert m.packed_rows(tokens, 16, 128) < 16 * 128
    outs = []
    for tok in (None, tokens):
        m.rng.zero_()
        m.zero_grad()
        loss, logits = m.forward_loss(ids, mask, labels, tokens=tok)
        loss.backward()
        torch.cuda.synchronize()
        outs.append((loss.detach().clone(), logits.clone(), m.arena.grad.clone(), m.emb_now.clone()))
    (l0, z0, g0, e0), (l1, z1, g1, e1) = outs
    assert rel(z1, z0) < 1e-3 and abs(float(l1 - l0)) < 1e-3
    # padded path also flags [PAD] (id 0, whose gradient is exactly 0); packed never sees it
    assert torch.equal(e0[1:], e1[1:]) and int(e1[0]) == 0
    dense = torch.ones_like(g0, dtype=torch.bool)
    woff, V, D = m.word_embedding_span()
    dense[woff:woff + V * D] = False
    assert rel(g1[dense], g0[dense]) < 2e-2
    assert not g0[woff:woff + D].any()  # the [PAD] row's padded-path gradient is exactly 0
    rows = e1.bool()
    assert rel(g1[woff:woff + V * D].view(V, D)[rows], g0[woff:woff + V * D].view(V, D)[rows]) < 2e-2


def test_packed_graph_buckets_match_eager():
    """Graph replays across batches of different real-token counts (one graph per bucket)
    track the eager packed path step for step."""
    cfg = DistilBertConfig(n_layers=2)
    models = [DDoSClassifier(config=cfg, device="cuda", impl="hip", seed=6) for _ in range(2)]
    steps = []
    for m, graph in zip(models, (True, False)):
        m.train()
        steps.append(GraphedTrainStep(make_step_fn(m, ArenaAdam(m, lr=1e-3)), warmup=1, enabled=graph,
                                      bucket=m.packed_rows))
    for it in range(6):
        lo, hi = ((40, 60), (70, 90), (40, 60))[it % 3]
        ids, mask, labels, tokens = _batch(16, 128, lo, hi, seed=50 + it)
        losses = [st(ids, mask, labels, tokens) for st in steps]
        torch.cuda.synchronize()
        assert abs(float(losses[0] - losses[1])) < 1e-5, it
    assert len(steps[0].graphs) >= 2 and steps[0].failed is None
    assert torch.equal(models[0].arena.master, models[1].arena.master)


@pytest.mark.parametrize("B,S", [(32, 128), (64, 256), (3, 64)])
def test_pack_kernel_matches_torch(B, S):
    """One-launch packing == nonzero / cumsum / gather in torch (prefix and holey masks)."""
    g = torch.Generator().manual_seed(B * S)
    lens = torch.randint(1, S + 1, (B,), generator=g)
    mask = (torch.arange(S)[None] < lens[:, None]).long()
    mask[1, 0] = 0 if B > 2 else mask[1, 0]  # a hole: the general (non-prefix) case still compacts
    ids = torch.randint(0, 30000, (B, S), generator=g)
    mask, ids = mask.cuda(), ids.cuda()
    total = int(mask.sum())
    rows = (total + 127) // 128 * 128
    row_map, cu, idp = K.pack(mask, ids, rows)
    ref_map = torch.nonzero(mask.reshape(-1)).squeeze(1)
    assert torch.equal(row_map[:total].long(), ref_map)
    assert (row_map[total:] == -1).all()
    ref_cu = torch.zeros(B + 1, dtype=torch.long)
    ref_cu[1:] = torch.cumsum(mask.sum(1).cpu(), 0)
    assert torch.equal(cu.cpu().long(), ref_cu)
    assert torch.equal(idp[:total], ids.reshape(-1)[ref_map])
    assert (idp[total:] == ids.reshape(-1)[0]).all()
    # a row budget smaller than the real tokens never writes past it
    small_map, _, _ = K.pack(mask, ids, 64)
    assert torch.equal(small_map.long(), ref_map[:64])


@pytest.mark.parametrize("S", [256, 512])
def test_long_sequence_model_hip_vs_torch(S):
    """the model at S = 256 / 512 (DistilBERT's position table caps S at 512),
    padded and packed HIP paths against the fp32 torch path, dropout on with identical masks."""
    cfg = DistilBertConfig(n_layers=2)
    hip = DDoSClassifier(config=cfg, device="cuda", impl="hip", seed=6)
    ref = DDoSClassifier(config=cfg, device="cuda", impl="torch", seed=6)
    ids, mask, labels, tokens = _batch(4, S, S // 3, S, seed=S)
    hip.train()
    ref.train()
    ref.rng.zero_() if hasattr(ref, "rng") else None
    ref.torch_counter = 0
    ref.zero_grad()
    lr_, zr = ref.forward_loss(ids, mask, labels)
    lr_.backward()
    g_ref = ref.arena.grad.clone()
    for tok in (None, tokens):
        hip.rng.zero_()
        hip.zero_grad()
        lh, zh = hip.forward_loss(ids, mask, labels, tokens=tok)
        lh.backward()
        torch.cuda.synchronize()
        assert rel(zh, zr) < 3e-2, (tok, rel(zh, zr))
        for name in ("distilbert.transformer.layer.0.attention.q_lin.weight",
                     "distilbert.transformer.layer.1.ffn.lin2.weight", "classifier.weight",
                     "distilbert.embeddings.position_embeddings.weight"):
            a, b = hip.dense_grad(name), ref.arena.gview(name)
            err = ((a - b).norm() / b.norm()).item()
            assert err < 3e-2, (tok, name, err)


def test_short_batch_attention_bitwise():
    """Every sequence <= 128 tokens at S = 256 (the caller's PackedTokens.max_len): the S <= 128
    kernels alone (split=2) give exactly what the length split gives (split=1) -- the skipped
    64-row launches had no sequence to take -- and the model step with a PackedTokens batch equals
    the one with a plain token count bit for bit, graph replay included."""
    from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.data import PackedTokens
    B, H, S = 8, 12, 256
    lens = torch.tensor([128, 77, 64, 1, 100, 65, 17, 16])
    n = int(lens.sum())
    g = torch.Generator(device="cuda").manual_seed(5)
    cu = torch.zeros(B + 1, dtype=torch.int32, device="cuda")
    cu[1:] = torch.cumsum(lens, 0).to(torch.int32).cuda()
    qkv = torch.cat([(torch.randn(n, 3 * H * 64, device="cuda", generator=g) * 0.5).to(torch.bfloat16),
                     torch.zeros(64, 3 * H * 64, dtype=torch.bfloat16, device="cuda")])
    dctx = torch.cat([(torch.randn(n, H * 64, device="cuda", generator=g) * 0.5).to(torch.bfloat16),
                      torch.zeros(64, H * 64, dtype=torch.bfloat16, device="cuda")])
    kb = K.mask_bias(torch.ones(B, S, dtype=torch.int64, device="cuda"))
    seed = torch.tensor([13], dtype=torch.int32, device="cuda")
    out = []
    for short in (False, True):
        ctx, lse = K.attn_fwd(qkv, kb, B, S, H, seed, 42, 0.1, cu=cu, short=short)
        d = K.attn_bwd(qkv, kb, ctx, lse, dctx, B, S, H, seed, 42, 0.1, cu=cu, short=short)
        out.append((ctx, d))
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])

    cfg = DistilBertConfig(n_layers=2)
    ids, mask, labels, tokens = _batch(16, S, 70, 90, seed=9)
    lmax = int(mask.sum(1).max())
    assert lmax <= 128
    res = []
    fused0 = K.ATTN_SHORT_FUSED
    try:
        # the S <= 128 producer-GEMM fusions in short mode (opt-in, FD_ATTN_SHORT_FUSED) are bitwise too
        for tok, graph, fused in ((tokens, False, False), (PackedTokens(tokens, lmax), False, False),
                                  (PackedTokens(tokens, lmax), True, False), (PackedTokens(tokens, lmax), False, True)):
            K.ATTN_SHORT_FUSED = fused
            m = DDoSClassifier(config=cfg, device="cuda", impl="hip", seed=8)
            m.train()
            st = GraphedTrainStep(make_step_fn(m, ArenaAdam(m, lr=1e-3)), warmup=1, enabled=graph,
                                  bucket=m.packed_rows)
            losses = [float(st(ids, mask, labels, tok)) for _ in range(3)]
            torch.cuda.synchronize()
            res.append((losses, m.arena.master.clone()))
    finally:
        K.ATTN_SHORT_FUSED = fused0
    assert res[0][0] == res[1][0] == res[2][0] == res[3][0]
    for r in res[1:]:
        assert torch.equal(res[0][1], r[1])
