"""Sweep every GEMM configuration on the DistilBERT training GEMMs (T tokens; the unpadded bs32 step
runs ~2.6-2.8 k packed rows, the padded one 4096).

For each of the 12 per-layer GEMMs (with the epilogue the model uses) and each
configuration id of csrc/kernels/gemm.hip (and split count for dW), time the
kernel with HIP events and check it against torch fp32.  Prints one line per
(gemm, cfg) and the best configuration per GEMM.

usage: python scripts/gemm_sweep.py [T=2688]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops._ext import ext

T = int(sys.argv[1]) if len(sys.argv) > 1 else 2688
NCFG = 25
g = torch.Generator(device="cuda").manual_seed(0)


def rnd(*s, scale=1.0):
    return ((torch.rand(*s, device="cuda", generator=g) * 2 - 1) * scale).to(torch.bfloat16)


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6)).item()


cases = []
# The model's current calls (ops/functional.py): forward NT (+bias / +bias+GELU), backward dX as NT
# on the transposed weight copy (+GELU' / +residual), weight gradients as grouped TN pairs.
W = {}
for name, N, Kd in [("qkv", 2304, 768), ("o", 768, 768), ("ffn1", 3072, 768), ("ffn2", 768, 3072)]:
    x, w, b = rnd(T, Kd), rnd(N, Kd, scale=0.05), torch.randn(N, device="cuda") * 0.1
    wt = w.t().contiguous()
    W[name] = (x, w, N, Kd)
    if name == "ffn1":
        ref = x.float() @ w.float().t() + b
        cases.append((f"{name}.fwd NT+gelu", 0, T * N * Kd, lambda x=x, w=w, b=b: K.linear_fwd(x, w, b, gelu=True)[1],
                      ref))
    else:
        cases.append((f"{name}.fwd NT+bias", 0, T * N * Kd, lambda x=x, w=w, b=b: K.linear_fwd(x, w, b),
                      x.float() @ w.float().t() + b))
    dy = rnd(T, N)
    res = rnd(T, Kd)
    if name == "ffn2":  # dX of lin2 carries gelu'(u) of lin1's pre-activation
        u = rnd(T, Kd)
        uu = u.float().requires_grad_(True)
        ref = torch.autograd.grad(torch.nn.functional.gelu(uu), uu, dy.float() @ w.float())[0]
        cases.append((f"{name}.dX NN+gelu'", 1, T * N * Kd,
                      lambda dy=dy, w=w, u=u: K.linear_dx(dy, w, gelu_u=u), ref))
    elif name in ("ffn1", "qkv"):
        cases.append((f"{name}.dX NN+add", 1, T * N * Kd,
                      lambda dy=dy, w=w, r=res: K.linear_dx(dy, w, res=r),
                      dy.float() @ w.float() + res.float()))
    else:
        cases.append((f"{name}.dX NN", 1, T * N * Kd, lambda dy=dy, w=w: K.linear_dx(dy, w),
                      dy.float() @ w.float()))
    W[name] = W[name] + (dy,)
for a, b_ in (("ffn2", "ffn1"), ("o", "qkv")):
    xa, wa, Na, Ka, dya = W[a]
    xb, wb, Nb, Kb, dyb = W[b_]
    oa, ob = torch.empty(Na, Ka, device="cuda"), torch.empty(Nb, Kb, device="cuda")
    ref = torch.cat([(dya.float().t() @ xa.float()).flatten(), (dyb.float().t() @ xb.float()).flatten()])

    def fn(dya=dya, xa=xa, oa=oa, dyb=dyb, xb=xb, ob=ob):
        K.linear_dw2(dya, xa, oa, dyb, xb, ob)
        return torch.cat([oa.flatten(), ob.flatten()])
    cases.append((f"{a}+{b_}.dW TN2", 2, T * (Na * Ka + Nb * Kb), fn, ref))

best = {}
for name, kind, macs, fn, ref in cases:
    opts = [(c, -1) for c in range(NCFG)] if kind != 2 else [(c, s) for c in range(NCFG) for s in (1, 2, 4, 8)]
    for cfg, sp in opts:
        try:
            ext().gemm_set_cfg(kind, cfg, sp)  # (ids not instantiated are rejected)
            out = fn()
            torch.cuda.synchronize()
        except RuntimeError as e:
            continue
        err = rel(out, ref)
        us = timeit(fn)
        ok = err < 2e-2
        tag = f"cfg={cfg:2d}" + (f" splits={sp}" if kind == 2 else "")
        print(f"{name:18s} {tag:18s} {us:8.1f} us {2 * macs / us / 1e6:6.0f} TF  err={err:.1e}{'' if ok else '  BAD'}",
              flush=True)
        if ok and (name not in best or us < best[name][0]):
            best[name] = (us, tag)
    ext().gemm_set_cfg(kind, -1, -1)
    us = timeit(fn)
    print(f"{name:18s} {'default':18s} {us:8.1f} us {2 * macs / us / 1e6:6.0f} TF", flush=True)
    best[name + " (default)"] = (us, "default")
print("\nbest per GEMM:")
tot_best = tot_def = 0.0
for k, (us, tag) in best.items():
    print(f"  {k:30s} {tag:18s} {us:8.1f} us")
    if k.endswith("(default)"):
        tot_def += us
    else:
        tot_best += us
print(f"sum best {tot_best:.1f} us/layer, sum default {tot_def:.1f} us/layer")
