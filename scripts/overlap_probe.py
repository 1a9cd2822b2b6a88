"""Do the all-layer dW GEMM (fp32 gradient stores, no Adam) and an HBM-bound Adam stream over
as many parameters overlap when they run side by side on two streams?  Times each alone and
both together (no dependency between them), isolated, at the packed bs32 step's shapes.

    python scripts/overlap_probe.py [T] [adam_blocks]
"""
import sys

import torch

sys.path.insert(0, ".")
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K  # noqa

T = int(sys.argv[1]) if len(sys.argv) > 1 else 2688
g = torch.Generator(device="cuda").manual_seed(0)
shapes = [(2304, 768), (768, 768), (3072, 768), (768, 3072)] * 6
jobs = []
for M, N in shapes:
    dy = (torch.randn(T, M, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
    x = torch.randn(T, N, device="cuda", generator=g).to(torch.bfloat16)
    jobs.append((dy, x, torch.empty(M, N, device="cuda"), False))
n = sum(M * N for M, N in shapes)
p, gr = torch.randn(n, device="cuda"), torch.randn(n, device="cuda") * 1e-3
m, v = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
sh = p.to(torch.bfloat16)
step = torch.ones(1, dtype=torch.int32, device="cuda")
s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()


def gemm():
    K.linear_dw_batch(jobs)


def adam():
    K.adam(p, gr, m, v, sh, step, 1e-5, 0.9, 0.999, 1e-8, 0.0, False)


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / iters


def both():
    cur = torch.cuda.current_stream()
    s0.wait_stream(cur)
    s1.wait_stream(cur)
    with torch.cuda.stream(s0):
        gemm()
    with torch.cuda.stream(s1):
        adam()
    cur.wait_stream(s0)
    cur.wait_stream(s1)


def both_rev():  # the Adam stream's kernel first
    cur = torch.cuda.current_stream()
    s0.wait_stream(cur)
    s1.wait_stream(cur)
    with torch.cuda.stream(s1):
        adam()
    with torch.cuda.stream(s0):
        gemm()
    cur.wait_stream(s0)
    cur.wait_stream(s1)


tg, ta = timed(gemm), timed(adam)
tb, tr = timed(both), timed(both_rev)
print(f"{n / 1e6:.1f} M params | dW GEMM alone {tg:7.1f} us | Adam alone {ta:7.1f} us | sum {tg + ta:7.1f} | "
      f"side by side {tb:7.1f} us (Adam launched second) / {tr:7.1f} us (first)")
