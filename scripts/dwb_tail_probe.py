"""Where the all-layer weight-gradient launch spends its time: isolated timings of problem SUBSETS
of the packed bs32 step's launch (fused Adam, as in the step), to expose its tile rounds.

The step's launch holds, in backward order, the pruned last block's lin2 / lin1 / out_lin weight
gradients (K = 64 [CLS] rows: 81 short 256 x 256 tiles), its qkv weight gradient (K = T, 27 long
tiles), then 4 x 108 long tiles for each of the other five blocks.  With the XCD remap each XCD
walks a contiguous 1/8 of the logical tile list, so XCD 0 gets the 81 short tiles and XCDs 1..7 get
81 long tiles each: 32 + 32 + 17 tiles per XCD, i.e. three rounds of long tiles, the third at
17/32 occupancy.  Usage: python scripts/dwb_tail_probe.py [T]"""
import sys

import torch

sys.path.insert(0, ".")
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K  # noqa

T = int(sys.argv[1]) if len(sys.argv) > 1 else 2688
g = torch.Generator(device="cuda").manual_seed(0)
LAYER = [(768, 3072), (3072, 768), (768, 768), (2304, 768)]  # lin2, lin1, out, qkv (backward order)


def make(Kt, M, N):
    dy = (torch.randn(Kt, M, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
    x = torch.randn(Kt, N, device="cuda", generator=g).to(torch.bfloat16)
    out = torch.empty(M, N, device="cuda")
    st = [torch.randn(M * N, device="cuda"), torch.zeros(M * N, device="cuda"), torch.zeros(M * N, device="cuda"),
          torch.empty(M * N, device="cuda", dtype=torch.bfloat16)]
    return (dy, x, out, False), st


pruned = [make(64, M, N) for M, N in LAYER[:3]] + [make(T, *LAYER[3])]
full = [[make(T, M, N) for M, N in LAYER] for _ in range(5)]
step = torch.ones(1, dtype=torch.int32, device="cuda")


def run(probs, fused=True, n=20):
    jobs = [p[0] for p in probs]
    states = [p[1] for p in probs]

    def adam(outs):
        st = []
        for s in states[:len(outs)]:
            st += s
        return st + [step], [2e-5, 0.9, 0.999, 1e-8, 0.0, 0.0]

    fn = lambda: K.linear_dw_batch(jobs, adam=adam if fused else None)  # noqa: E731
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def tiles(probs):
    return sum((p[0][0].shape[1] // 256) * (p[0][1].shape[1] // 256) for p in probs)


flat = [p for layer in full for p in layer]
sets = [
    ("step order (pruned first), 24 problems", pruned + flat),
    ("pruned block last", flat + pruned),
    ("reversed (forward block order)", (pruned + flat)[::-1]),
    ("reversed blocks, backward order inside", [p for layer in full[::-1] for p in layer] + pruned),
    ("5 long blocks only", flat),
    ("pruned block only (81 short + 27 long)", pruned),
    ("pruned short only (81 tiles, K=64)", pruned[:3]),
    ("one long block (108 tiles)", full[0]),
    ("two long blocks (216)", full[0] + full[1]),
    ("three long blocks (324)", full[0] + full[1] + full[2]),
    ("four long blocks (432)", [p for layer in full[:4] for p in layer]),
]
for name, probs in sets:
    a = run(probs, True)
    b = run(probs, False)
    print(f"{name:42s} tiles {tiles(probs):4d}  fused-Adam {a:7.1f} us   no-Adam {b:7.1f} us", flush=True)
