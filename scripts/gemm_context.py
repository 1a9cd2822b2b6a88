"""Does a GEMM run slower inside the training step than alone?  Time the FFN2
forward (M=4096, N=768, K=3072, bias) (a) back to back, (b) right after the FFN1
forward that produces its input, (c) after a 512 MB write that evicts L2/MALL."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K  # noqa: E402,E501

T = 4096
g = torch.Generator(device="cuda").manual_seed(0)


def rnd(*s):
    return (torch.randn(*s, device="cuda", generator=g) * 0.1).to(torch.bfloat16)


x, w1, b1 = rnd(T, 768), rnd(3072, 768), torch.zeros(3072, device="cuda")
w2, b2 = rnd(768, 3072), torch.zeros(768, device="cuda")
w2t = w2.t().contiguous()
dz = rnd(T, 768)
flush = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
gg, u = K.linear_fwd(x, w1, b1, gelu=True)


def timed(pre, fn, iters=30):
    es = []
    for i in range(iters + 3):
        pre()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        es.append((e0, e1))
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in es[3:])
    return ts[len(ts) // 2]


nop = lambda: None  # noqa: E731
ffn1 = lambda: K.linear_fwd(x, w1, b1, gelu=True)  # noqa: E731
fl = lambda: flush.fill_(1)  # noqa: E731
ffn2 = lambda: K.linear_fwd(gg, w2, b2)  # noqa: E731
l1dx = lambda: K.linear_dx(gg, w2t, res=dz)  # noqa: E731  (dh = du W1 + dz: K=3072, N=768)
for name, fn in (("ffn2 fwd", ffn2), ("l1 dX+res", l1dx)):
    a = timed(nop, fn)
    b = timed(ffn1, fn)
    c = timed(fl, fn)
    fla = 2 * T * 768 * 3072 / 1e6
    print(f"{name:10s} alone {a:6.1f} us ({fla / a:4.0f} TF) | after ffn1 {b:6.1f} us | after 512MB write {c:6.1f} us",
          flush=True)
