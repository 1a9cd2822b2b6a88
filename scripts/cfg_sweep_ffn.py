"""Tile-configuration sweep of the FFN GEMMs at the packed bs32 step's shape (M = 2688 rows):
FFN1 forward (NT, bias + GELU epilogue, N = 3072, K = 768) and the FFN2 dX with the GELU'
epilogue (NN on W, + gelu(u) re-creation + lin1 bias column sums, N = 3072, K = 768), per
instantiated configuration id (csrc/kernels/gemm.hip CFGS), against torch.matmul (hipBLASLt).

    python scripts/cfg_sweep_ffn.py [M] [cfgs]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K  # noqa: E402,E501


def timeit(fn, iters=100):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / iters


M = int(sys.argv[1]) if len(sys.argv) > 1 else 2688
cfgs = [int(c) for c in (sys.argv[2] if len(sys.argv) > 2 else "-1,0,1,3,6,8,10,18,21,24").split(",")]
g = torch.Generator(device="cuda").manual_seed(0)
D, F = 768, 3072
x = torch.randn(M, D, device="cuda", generator=g).to(torch.bfloat16)
w1 = (torch.randn(F, D, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
b1 = torch.randn(F, device="cuda", generator=g) * 0.1
w2 = (torch.randn(D, F, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
dy = torch.randn(M, D, device="cuda", generator=g).to(torch.bfloat16)
u = torch.randn(M, F, device="cuda", generator=g).to(torch.bfloat16)
gout = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
db1 = torch.zeros(F, device="cuda")
fl = 2.0 * M * F * D
t_ref = timeit(lambda: torch.nn.functional.linear(x, w1))
t_ref2 = timeit(lambda: dy @ w2)
print(f"torch (hipBLASLt, bare matmul): ffn1 fwd {t_ref:6.1f} us {fl / t_ref / 1e6:5.0f} TF | "
      f"ffn2 dX {t_ref2:6.1f} us {fl / t_ref2 / 1e6:5.0f} TF", flush=True)
for c in cfgs:
    try:
        K.ext().gemm_set_cfg(0, c, -1)
        K.ext().gemm_set_cfg(1, c, -1)
    except RuntimeError:
        print(f"cfg {c:3d}: not instantiated", flush=True)
        continue
    t1 = timeit(lambda: K.linear_fwd(x, w1, b1, gelu=True))

    def dx():
        jobs = []
        K.linear_dx(dy, w2, gelu_u=u, colsum=(jobs, db1, False), aux_out=gout)
        K.colsum_flush(jobs)
    t2 = timeit(dx)
    print(f"cfg {c:3d}: ffn1 fwd (bias+GELU) {t1:6.1f} us {fl / t1 / 1e6:5.0f} TF | "
          f"ffn2 dX (GELU' + gelu + colsum) {t2:6.1f} us {fl / t2 / 1e6:5.0f} TF", flush=True)
K.ext().gemm_set_cfg(0, -1, -1)
K.ext().gemm_set_cfg(1, -1, -1)
