"""Where does the HIP path drift from the fp32 torch path over training? (loss-curve bias hunt)
1. stale-gradient check: HIP grads of batch B after an unrelated backward of batch A (zero_grad in
   between) vs a fresh model on batch B -- must be bitwise equal.
2. parameter drift: HIP and torch trained on the same batches (dropout off, eager), per tensor
   ||p_hip - p_torch|| / ||p_torch - p_0|| after 1 / 10 / 50 steps (top tensors), and the same
   ratio for the torch path under bf16 autocast as a noise yardstick."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.data import (  # noqa: E402
    DeviceLoader, build_client_data, generate_cicids2017)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.engine import (  # noqa: E402
    ArenaAdam, make_step_fn)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.models import (  # noqa: E402
    DDoSClassifier, DistilBertConfig)


def model(impl):
    cfg = DistilBertConfig(dropout=0.0, attention_dropout=0.0)
    m = DDoSClassifier(config=cfg, device="cuda", impl=impl, seed=8, head_dropout=0.0)
    m.train()
    return m


def main():
    frame = generate_cicids2017(8000, seed=5, hard=True)
    cd = build_client_data(frame, 0, data_fraction=1.0, max_len=128)
    batches = list(DeviceLoader(cd.train, 32, shuffle=True, device="cuda", seed=3, drop_last=True))[:60]
    names = list(model("torch").state_dict().keys())

    # 1. stale gradients
    a, b = batches[0], batches[1]
    m1 = model("hip")
    m1.zero_grad(); l, _ = m1.forward_loss(a["input_ids"], a["attention_mask"], a["labels"]); l.backward()
    m1.zero_grad(); l, _ = m1.forward_loss(b["input_ids"], b["attention_mask"], b["labels"]); l.backward()
    m2 = model("hip")
    m2.zero_grad(); l, _ = m2.forward_loss(b["input_ids"], b["attention_mask"], b["labels"]); l.backward()
    torch.cuda.synchronize()
    bad = [n for n in names if not torch.equal(m1.dense_grad(n), m2.dense_grad(n))]
    print(f"stale-gradient check: {len(bad)} tensors differ {bad[:8]}", flush=True)
    del m1, m2

    # 2. drift
    def run(impl, autocast=False):
        m = model(impl)
        opt = ArenaAdam(m, lr=2e-5)
        fn = make_step_fn(m, opt)
        snaps = {0: {n: m.arena.view(n).detach().clone() for n in names}}
        for i, bt in enumerate(batches[:50]):
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
                fn(bt["input_ids"], bt["attention_mask"], bt["labels"], None)
            if i + 1 in (1, 10, 50):
                torch.cuda.synchronize()
                snaps[i + 1] = {n: m.arena.view(n).detach().clone() for n in names}
        del opt, fn, m
        torch.cuda.empty_cache()
        return snaps
    sh, st, sb = run("hip"), run("torch"), run("torch", autocast=True)
    for k in (1, 10, 50):
        rows = []
        for n in names:
            upd = (st[k][n] - st[0][n]).float().norm().item()
            if upd == 0:
                continue
            rows.append(((sh[k][n] - st[k][n]).float().norm().item() / upd,
                         (sb[k][n] - st[k][n]).float().norm().item() / upd, n))
        rows.sort(reverse=True)
        tot_h = sum(r[0] for r in rows) / len(rows)
        tot_b = sum(r[1] for r in rows) / len(rows)
        print(f"after {k} steps: mean over tensors hip {tot_h:.3f} autocast {tot_b:.3f};  top ||hip - torch|| / "
              f"||torch update|| (autocast torch alongside):", flush=True)
        for r in rows[:12]:
            print(f"   {r[0]:.3f}  (autocast {r[1]:.3f})  {r[2]}")
        # signed: does the HIP update run AHEAD of torch's along torch's own direction?
        ahead = []
        for n in names:
            dt = (st[k][n] - st[0][n]).float().flatten()
            if dt.norm() == 0:
                continue
            dh = (sh[k][n] - st[0][n]).float().flatten()
            db = (sb[k][n] - st[0][n]).float().flatten()
            ahead.append(((dh.norm() / dt.norm()).item(), (db.norm() / dt.norm()).item(), n))
        ahead.sort(reverse=True)
        print(f"   update-norm ratio hip/torch: top {[(round(a, 3), round(b, 3), n) for a, b, n in ahead[:6]]}")
        print(f"   update-norm ratio hip/torch: bottom {[(round(a, 3), round(b, 3), n) for a, b, n in ahead[-4:]]}")


if __name__ == "__main__":
    main()
