"""How much of a step GEMM's in-step time is cold operands?  Times the QKV forward GEMM
(M = 2688, N = 2304, K = 768) and the out-proj LayerNorm-fused forward with every operand hot
(back-to-back repeats), with the weight evicted from L2 / MALL before each call (a 1 GiB
streaming write in between), and with the activation evicted instead.

    python scripts/cold_weight_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K  # noqa: E402,E501

M, D = 2688, 768
g = torch.Generator(device="cuda").manual_seed(0)
flush = torch.empty(256 << 20, device="cuda")  # 1 GiB: well past the 256 MiB MALL


def timed(fn, evict=None, iters=30):
    ts = []
    for i in range(iters + 3):
        if evict is not None:
            evict()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        if i >= 3:
            ts.append(a.elapsed_time(b) * 1000)
    ts.sort()
    return ts[len(ts) // 2]


def evict_all():
    flush.fill_(1.0)


for name, N in (("qkv fwd", 3 * D), ("ffn1 fwd", 4 * D)):
    x = torch.randn(M, D, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(N, D, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device="cuda", generator=g) * 0.1
    fn = (lambda: K.linear_fwd(x, w, b)) if N == 3 * D else (lambda: K.linear_fwd(x, w, b, gelu=True))

    def warm_x():  # everything cold, then the activation re-read (as if just produced)
        evict_all()
        x.add_(0)

    def warm_w():
        evict_all()
        w.add_(0)

    hot = timed(fn)
    cold = timed(fn, evict_all)
    wcold = timed(fn, warm_x)
    xcold = timed(fn, warm_w)
    print(f"{name:8s}: hot {hot:6.1f} us | all cold {cold:6.1f} | weight cold (activation warm) {wcold:6.1f} | "
          f"activation cold (weight warm) {xcold:6.1f}", flush=True)
