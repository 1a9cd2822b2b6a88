"""Can two ranks run RCCL collectives on ONE GPU?  (The pool gives one MI355X per box; the native
RCCL module csrc/comm/rccl_comm.cpp has only ever run single-rank.)  Two spawned processes, both on
cuda:0: a gloo torch.distributed group for the unique-id rendezvous, then NativeComm all-reduce
(sum / avg), broadcast and all-gather against exact values.  Prints one JSON line per rank and a
verdict; every step is bounded (NativeComm's own wait, and the caller's timeout).

    python scripts/rccl_one_gpu_probe.py [outdir]
"""
import json
import os
import socket
import sys
import traceback

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = "detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd"


def _worker(rank, world, port, outdir):
    res = {"rank": rank}
    try:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from importlib import import_module
        NativeComm = import_module(f"{PKG}.parallel.rccl").NativeComm
        c = NativeComm(timeout_s=30.0)
        res["init"] = True
        x = torch.arange(1 << 20, dtype=torch.float32, device="cuda") * (rank + 1)
        base = torch.arange(1 << 20, dtype=torch.float32, device="cuda")
        c.all_reduce_(x, "sum")
        res["sum"] = torch.equal(x, base * sum(r + 1 for r in range(world)))
        y = torch.full((4096,), float(2 * rank + 1), device="cuda")
        c.all_reduce_(y, "avg")
        res["avg"] = torch.equal(y, torch.full_like(y, float(world)))
        z = torch.full((1000,), float(rank + 7), device="cuda").to(torch.bfloat16)
        c.broadcast_(z, root=1)
        res["bcast"] = torch.equal(z, torch.full_like(z, 8.0))
        g = c.all_gather(torch.full((16,), float(rank), device="cuda"))
        res["gather"] = all(torch.equal(g[r], torch.full((16,), float(r), device="cuda")) for r in range(world))
        # a 265 MB all-reduce (the FedAvg payload) timed with events
        big = torch.ones(265_000_000 // 4, dtype=torch.float32, device="cuda")
        c.all_reduce_(big, "sum")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            c.all_reduce_(big, "sum", wait=False)
        e1.record()
        c.wait("timed all_reduce")
        res["allreduce_265MB_ms"] = round(e0.elapsed_time(e1) / 3, 3)
        torch.cuda.synchronize()
        c.close()
    except Exception as e:  # noqa: BLE001 -- the probe reports whatever RCCL says
        res["error"] = f"{type(e).__name__}: {e}"
        res["trace"] = traceback.format_exc()[-1500:]
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    try:
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        pass


def main():
    outdir = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/rccl_probe"
    os.makedirs(outdir, exist_ok=True)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_worker, args=(2, port, outdir), nprocs=2, join=True)
    out = [json.load(open(os.path.join(outdir, f"rank{r}.json"))) for r in range(2)]
    for r in out:
        print(json.dumps({k: v for k, v in r.items() if k != "trace"}))
    ok = all(r.get(k) for r in out for k in ("init", "sum", "avg", "bcast", "gather"))
    print("verdict:", "two RCCL ranks on one GPU work" if ok else "not supported / failed (see errors)")


if __name__ == "__main__":
    main()
