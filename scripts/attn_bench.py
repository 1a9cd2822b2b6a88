"""Time the attention kernels (varlen, ~80-token sequences, S=128) at several batch sizes:
constant time across B = per-block latency bound, linear = throughput bound."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K  # noqa: E402,E501


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


S, H = 128, 12
g = torch.Generator(device="cuda").manual_seed(0)
seed = torch.tensor([3], dtype=torch.int32, device="cuda")
for B in (1, 4, 16, 32, 64, 128):
    lens = torch.randint(76, 87, (B,), generator=torch.Generator().manual_seed(B))
    cu = torch.zeros(B + 1, dtype=torch.int32)
    cu[1:] = torch.cumsum(lens, 0)
    cu = cu.cuda()
    rows = (int(lens.sum()) + 127) // 128 * 128
    qkv = (torch.randn(rows, 3 * H * 64, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    kb = torch.zeros(B * S, device="cuda")
    dctx = (torch.randn(rows, H * 64, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    for p, bits in ((0.0, False), (0.1, False), (0.1, True)):
        dm = K.attn_keep_bits(B, S, H, p, "cuda") if bits else None
        ctx, lse = K.attn_fwd(qkv, kb, B, S, H, seed, 5, p, cu=cu, dmask=dm)
        tf = timeit(lambda: K.attn_fwd(qkv, kb, B, S, H, seed, 5, p, cu=cu, dmask=dm))
        tb = timeit(lambda: K.attn_bwd(qkv, kb, ctx, lse, dctx, B, S, H, seed, 5, p, cu=cu, dmask=dm))
        print(f"S128={os.environ.get('FD_ATTN_S128', '1')} B={B:4d} p={p} keep-bits={int(bits)}: fwd {tf:7.1f} us  "
              f"bwd {tb:7.1f} us", flush=True)
