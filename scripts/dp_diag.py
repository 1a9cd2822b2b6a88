"""Diag: sum of two half-batch HIP gradients vs the full-batch gradient (test_dp_gpu's check,
in one process), worst tensors and word-embedding rows."""
import sys, os
sys.path.insert(0, os.getcwd())
import torch
sys.path.insert(0, "tests")
from test_dp_gpu import _batch, _model

dev = torch.device("cuda")
ids, mask, labels = _batch(dev)
def run(sl, scale):
    m = _model(dev)
    m.zero_grad()
    loss, _ = m.forward_loss(ids[sl], mask[sl], labels[sl])
    (loss * scale).backward()
    torch.cuda.synchronize()
    return m, m.arena.grad.clone(), m.emb_now.clone()
m, g0, n0 = run(slice(0, 8), 0.5)
_, g1, n1 = run(slice(8, 16), 0.5)
_, gf, nf = run(slice(0, 16), 1.0)
woff, V, D = m.word_embedding_span()
gs = g0 + g1
w0, w1 = g0[woff:woff + V * D].view(V, D), g1[woff:woff + V * D].view(V, D)
gs[woff:woff + V * D] = (w0 * n0[:, None].to(w0.dtype) + w1 * n1[:, None].to(w1.dtype)).reshape(-1)
rows = nf.bool()
gw, rw = gs[woff:woff + V * D].view(V, D)[rows], gf[woff:woff + V * D].view(V, D)[rows]
d = (gw - rw).abs()
i = int(d.max(1).values.argmax())
ridx = rows.nonzero().squeeze(1)[i].item()
print(f"word rows: max abs {d.max().item():.3e} at vocab row {ridx}; row norm ref {rw[i].norm().item():.3e} "
      f"diff {(gw[i]-rw[i]).norm().item():.3e}; overall rel {((gw-rw).norm()/rw.norm()).item():.3e}")
errs = []
for k in m.state_dict():
    a = m.arena.gview(k)
    off = a.data_ptr() - m.arena.grad.data_ptr()
    n = a.numel(); o = off // 4
    x, y = gs[o:o + n], gf[o:o + n]
    if y.norm() > 0:
        errs.append((((x - y).norm() / y.norm()).item(), k))
for e, k in sorted(errs, reverse=True)[:8]:
    print(f"  {e:.3e} {k}")
