"""Run one GEMM shape/kind/epilogue N times (rocprofv3 PMC collection, timing A/B).

usage: gemm_one.py {nt,nt_gelu,nt_plain,nn,nn_gelu,nn_add,tn} M N K [iters]
FD_GEMM_TILE / FD_GEMM_VARIANT / FD_GEMM_GROUP_M select the kernel.
Prints the mean time per call (HIP events) so the same run serves as a timing probe.
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K

kind, M, N, Kd = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
it = int(sys.argv[5]) if len(sys.argv) > 5 else 20
g = torch.Generator(device="cuda").manual_seed(0)
rnd = lambda *s: (torch.rand(*s, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
b = torch.randn(N, device="cuda")
if kind.startswith("nt"):
    x, w = rnd(M, Kd), rnd(N, Kd)
    fn = {"nt": lambda: K.linear_fwd(x, w, b), "nt_gelu": lambda: K.linear_fwd(x, w, b, gelu=True),
          "nt_plain": lambda: K.linear_fwd(x, w, None)}[kind]
elif kind.startswith("nn"):
    dy, w = rnd(M, Kd), rnd(Kd, N)
    u = rnd(M, N)
    fn = {"nn": lambda: K.linear_dx(dy, w), "nn_gelu": lambda: K.linear_dx(dy, w, gelu_u=u),
          "nn_add": lambda: K.linear_dx(dy, w, res=u)}[kind]
else:
    # dW[M][N] = dy^T x with dy [Kd, M], x [Kd, N]
    dy, x = rnd(Kd, M), rnd(Kd, N)
    out = torch.empty(M, N, device="cuda")
    fn = lambda: K.linear_dw(dy, x, out)
for _ in range(3):
    fn()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(it):
    fn()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / it * 1e3
print(f"{kind} M={M} N={N} K={Kd} tile={os.environ.get('FD_GEMM_TILE', 'auto')}: {us:.1f} us "
      f"{2 * M * N * Kd / us / 1e6:.0f} TF", flush=True)
