"""Attention kernels alone at the bs32 packed shape (for rocprofv3 --pmc passes):
50 forward + 50 backward launches, p = 0.1 with the forward's keep bits."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K  # noqa: E402,E501

B, S, H = 32, 128, 12
g = torch.Generator(device="cuda").manual_seed(0)
seed = torch.tensor([3], dtype=torch.int32, device="cuda")
lens = torch.randint(76, 87, (B,), generator=torch.Generator().manual_seed(B))
cu = torch.zeros(B + 1, dtype=torch.int32)
cu[1:] = torch.cumsum(lens, 0)
cu = cu.cuda()
rows = (int(lens.sum()) + 127) // 128 * 128
qkv = (torch.randn(rows, 3 * H * 64, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
kb = torch.zeros(B * S, device="cuda")
dctx = (torch.randn(rows, H * 64, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
dm = K.attn_keep_bits(B, S, H, 0.1, "cuda")
for _ in range(50):
    ctx, lse = K.attn_fwd(qkv, kb, B, S, H, seed, 5, 0.1, cu=cu, dmask=dm)
for _ in range(50):
    K.attn_bwd(qkv, kb, ctx, lse, dctx, B, S, H, seed, 5, 0.1, cu=cu, dmask=dm)
torch.cuda.synchronize()
print("ok")
