"""Run one GEMM shape/kind N times (for rocprofv3 PMC collection)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K
kind, M, N, Kd = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
it = int(sys.argv[5]) if len(sys.argv) > 5 else 20
x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
w = torch.randn(N, Kd, device="cuda").to(torch.bfloat16)
b = torch.randn(N, device="cuda")
for _ in range(it):
    if kind == "nt":
        K.linear_fwd(x, w, b)
    elif kind == "nn":
        K.linear_dx(x, w.t().contiguous() if False else torch.randn(Kd, N, device="cuda").to(torch.bfloat16))
    else:
        out = torch.empty(N, Kd, device="cuda")
        K.linear_dw(torch.randn(M, N, device="cuda").to(torch.bfloat16), x, out)
torch.cuda.synchronize()
