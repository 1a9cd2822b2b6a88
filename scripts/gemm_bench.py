"""Time the framework's GEMM kernels vs torch.matmul (hipBLASLt) on the DistilBERT training shapes."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K

def timeit(fn, iters=50):
    for _ in range(5): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us

T = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
g = torch.Generator(device="cuda").manual_seed(0)
def rnd(*s): return torch.randn(*s, device="cuda", generator=g).to(torch.bfloat16)
rows = []
for (N, Kd, name) in [(2304, 768, "qkv"), (768, 768, "o"), (3072, 768, "ffn1"), (768, 3072, "ffn2")]:
    x, w, b = rnd(T, Kd), rnd(N, Kd), torch.randn(N, device="cuda")
    fl = 2 * T * N * Kd
    t_ours = timeit(lambda: K.linear_fwd(x, w, b, gelu=(name == "ffn1")))
    t_ref = timeit(lambda: torch.nn.functional.linear(x, w))
    dy = rnd(T, N)
    t_nn = timeit(lambda: K.linear_dx(dy, w))  # NN: W read MN-major (transposing LDS reads), no W^T copy
    t_nn_ref = timeit(lambda: dy @ w)
    out = torch.empty(N, Kd, device="cuda")
    t_tn = timeit(lambda: K.linear_dw(dy, x, out))
    t_tn_ref = timeit(lambda: dy.t() @ x)
    for kind, to, tr in [("NT fwd", t_ours, t_ref), ("dX", t_nn, t_nn_ref), ("TN dW", t_tn, t_tn_ref)]:
        rows.append((to, tr))
        print(f"{name:5s} {kind:7s} M={T} N={N} K={Kd}: ours {to:7.1f}us {fl/to/1e6:6.0f} TF | torch {tr:7.1f}us {fl/tr/1e6:6.0f} TF", flush=True)
print(f"per layer: ours {sum(r[0] for r in rows):.1f} us (fused epilogues) | torch {sum(r[1] for r in rows):.1f} us (bare matmuls)")
