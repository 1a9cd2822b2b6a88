"""Tile-configuration sweep of the QKV projection (NT, bias epilogue, N = 2304, K = 768) at a given row
count, per instantiated configuration id (csrc/kernels/gemm.hip CFGS), against torch (hipBLASLt).

    python scripts/cfg_sweep_qkv.py [M] [cfgs]
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


M = int(sys.argv[1]) if len(sys.argv) > 1 else 5184
cfgs = [int(c) for c in (sys.argv[2] if len(sys.argv) > 2 else "-1,0,1,3,6,8,10,18,21,24").split(",")]
g = torch.Generator(device="cuda").manual_seed(0)
D, N = 768, 2304
x = torch.randn(M, D, device="cuda", generator=g).to(torch.bfloat16)
w = (torch.randn(N, D, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
b = torch.randn(N, device="cuda", generator=g) * 0.1
fl = 2.0 * M * N * D
bb = b.to(torch.bfloat16)
t_ref = timeit(lambda: torch.nn.functional.linear(x, w, bb))
print(f"torch (hipBLASLt): qkv {t_ref:6.1f} us {fl / t_ref / 1e6:5.0f} TF", flush=True)
for c in cfgs:
    try:
        K.ext().gemm_set_cfg(0, c, -1)
    except RuntimeError:
        print(f"cfg {c:3d}: not instantiated", flush=True)
        continue
    t = timeit(lambda: K.linear_fwd(x, w, b))
    print(f"cfg {c:3d}: qkv fwd (bias) {t:6.1f} us {fl / t / 1e6:5.0f} TF", flush=True)
K.ext().gemm_set_cfg(0, -1, -1)
