"""Row-independence check of the N = 768 / 3072 GEMMs at M = 64 vs M = 2688 (pruned-block diagnostics)."""
import sys, torch
sys.path.insert(0, ".")
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K
torch.manual_seed(0)
T, D, F = 2688, 768, 3072
dev = "cuda"
bf = lambda *s, sc=1.0: (torch.randn(*s, device=dev) * sc).to(torch.bfloat16)
cx, x = bf(T, D), bf(T, D)
ow, ob = bf(D, D, sc=0.03), torch.randn(D, device=dev) * 0.1
g1, b1 = torch.ones(D, device=dev), torch.zeros(D, device=dev)
l1w, l1b = bf(F, D, sc=0.03), torch.randn(F, device=dev) * 0.1
seed = torch.tensor([3], dtype=torch.int32, device=dev)
ci = torch.arange(64, device=dev) * 40
h_full, *_ = K.linear_ln_fwd(cx, ow, ob, x, g1, b1, 1e-12, seed, 0, 0.0, keep_z=False)
h_p, *_ = K.linear_ln_fwd(cx.index_select(0, ci), ow, ob, x.index_select(0, ci), g1, b1, 1e-12, seed, 0, 0.0, keep_z=False)
print("ln-gemm rows equal:", torch.equal(h_full.index_select(0, ci), h_p), (h_full.index_select(0, ci).float() - h_p.float()).abs().max().item())
y_full = K.linear_fwd(h_full, l1w, l1b)
y_p = K.linear_fwd(h_full.index_select(0, ci), l1w, l1b)
print("ffn1 rows equal:", torch.equal(y_full.index_select(0, ci), y_p), (y_full.index_select(0, ci).float() - y_p.float()).abs().max().item())
g_full, u_full = K.linear_fwd(h_full, l1w, l1b, gelu=True)
g_p, u_p = K.linear_fwd(h_full.index_select(0, ci), l1w, l1b, gelu=True)
print("ffn1 gelu rows equal:", torch.equal(g_full.index_select(0, ci), g_p), (g_full.index_select(0, ci).float() - g_p.float()).abs().max().item())
l2w, l2b = bf(D, F, sc=0.03), torch.randn(D, device=dev) * 0.1
z_full, *_ = K.linear_ln_fwd(g_full, l2w, l2b, h_full, g1, b1, 1e-12, seed, 7, 0.0, keep_z=False)
z_p, *_ = K.linear_ln_fwd(g_full.index_select(0, ci), l2w, l2b, h_full.index_select(0, ci), g1, b1, 1e-12, seed, 7, 0.0, keep_z=False)
print("ln2-gemm rows equal:", torch.equal(z_full.index_select(0, ci), z_p), (z_full.index_select(0, ci).float() - z_p.float()).abs().max().item())
