"""Phase timing of the S <= 128 attention kernels from in-kernel stamps (diagnostic build).

    FD_BUILD_TAG=astamps FD_SO_OUT=ab/astamps.so FD_HIP_EXTRA_FLAGS=-DFD_ATTN_STAMPS=1 \\
        python -m <pkg>._build
    FD_SO_OUT=ab/astamps.so python scripts/attn_stamps.py [B]

Wave 0 of each (sequence, head) block stamps (attention.hip ASTAMP, 10 ns ticks):
fwd 0 entry, 1 staged (barrier), 2 softmax/PV loop done, 3 stored;
bwd 0 entry, 1 staged, 2 phase 1 (dQ) done, 3 phase-1 barrier, 4 phase 2 (dK/dV) stored.
Printed: median / max over blocks of each phase (us) relative to the block's entry, the
spread of entries, and the last exit."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K  # noqa: E402,E501
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops._ext import ext  # noqa: E402,E501


def report(name, nblocks, nph):
    st = torch.zeros(nblocks, 8, dtype=torch.int64)
    if ext().attn_stamps(st) < 0:
        print("not an attention-stamps build")
        sys.exit(1)
    t = st[:, :nph].double() / 100.0
    t = t - t[:, 0].min()
    hw = st[:, 7]
    cu = ((hw >> 32) << 8) | ((hw >> 8) & 0xff)
    _, counts = torch.unique(cu, return_counts=True)

    def q(x):
        return f"{x.median().item():6.2f}/{x.max().item():6.2f}"
    parts = [f"entry {q(t[:, 0])}"] + [f"ph{i} {q(t[:, i] - t[:, i - 1])}" for i in range(1, nph)]
    print(f"{name:10s} blocks {nblocks:4d} CUs {len(counts):3d} (max {counts.max().item()}/CU) | " + " | ".join(parts)
          + f" | exit {q(t[:, nph - 1])}", flush=True)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    S, H = 128, 12
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
    nblk = B * H  # (the filler-zeroing slice z == B comes after: not reported)
    for rep in range(2):
        for _ in range(20):
            ctx, lse = K.attn_fwd(qkv, kb, B, S, H, seed, 5, 0.1, cu=cu, dmask=dm)
        torch.cuda.synchronize()
        report(f"fwd B={B}", nblk, 4)
        for _ in range(20):
            K.attn_bwd(qkv, kb, ctx, lse, dctx, B, S, H, seed, 5, 0.1, cu=cu, dmask=dm)
        torch.cuda.synchronize()
        report(f"bwd B={B}", nblk, 5)


if __name__ == "__main__":
    main()
