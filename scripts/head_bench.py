"""Isolated timing of the pruned step's fused head + output-LN backward launch (norm.hip
head_ln_bwd_kernel) at the bench shapes (B = 32 [CLS] rows, T = 64 pruned rows, D = 768), with
and without the head / LN dropout, against the three launches it replaced."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.ops import kernels as K  # noqa: E402


def timeit(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / n


def main():
    dev = "cuda"
    B, T, D = 32, 64, 768
    g = torch.Generator(device="cpu").manual_seed(0)
    hidden = torch.randn(T, D, generator=g).to(torch.bfloat16).to(dev)
    z = torch.randn(T, D, generator=g).to(torch.bfloat16).to(dev)
    W = (torch.randn(2, D, generator=g) * 0.02).to(dev)
    b = torch.zeros(2, device=dev)
    labels = torch.randint(0, 2, (B,), generator=g).to(dev)
    seed = torch.tensor([5], dtype=torch.int32, device=dev)
    gamma = torch.ones(D, device=dev)
    mean, rstd = torch.zeros(T, device=dev), torch.ones(T, device=dev)
    dW, db = torch.zeros(2, D, device=dev), torch.zeros(2, device=dev)
    dgamma, dbeta, dbias = (torch.zeros(D, device=dev) for _ in range(3))
    rmap = torch.arange(T, dtype=torch.int32, device=dev)
    for ph, p in ((0.3, 0.1), (0.0, 0.1), (0.3, 0.0), (0.0, 0.0)):
        jobs = []

        def run():
            jobs.clear()
            K.head_ln_bwd(hidden, B, W, b, seed, 7, ph, labels, dW, db, False, None, z, gamma, mean, rstd, 9, p,
                          rmap, dgamma, dbeta, dbias, False, jobs)
        print(f"head_ln_bwd  p_head {ph} p_ln {p}: {timeit(run):6.2f} us/launch", flush=True)


if __name__ == "__main__":
    main()
