#!/usr/bin/env python3
"""Headline benchmark: local federated-client training throughput + aggregated F1.

Metric (BASELINE.json): batches/sec/client of DistilBERT-base DDoSClassifier
training at seq_len 128, batch 32, bf16 compute, on synthetic CICIDS2017-shaped
flows rendered to text (random-init weights), one client per GPU -- plus the
aggregated test F1 after 3 local epochs + 1 FedAvg round.

Two phases, one process per GPU:

1. Throughput (timed).  A "step" is the full reference step (client1.py:102-112):
   forward, CE loss, backward, Adam update -- here the fused HIP kernels replayed
   as a HIP graph.  W untimed warmup steps, then EXACTLY K timed steps between a
   barrier + device sync on both sides; the time is the MAX over ranks.  For N > 1
   every rank is an independent federated client and the timed region also ends
   with one FedAvg round (RCCL all-reduce of the 66.4 M fp32 masters), i.e. the
   communication is charged once per K steps (the reference averages once per 3
   epochs = 1,270 steps at bs32, so this over-charges it).  The batches are the
   client's real training split (below).
2. Quality (untimed, after the timed window).  The real BASELINE.json config-2/3
   protocol through the framework's own federated client (fed/runner.py):
   a 225,745-row synthetic CICIDS2017 file, a 10 % sample per client (seed
   42 + client), 60/20/20 split (13,544 / 4,515 / 4,515 rows), 3 local epochs of
   Adam lr 2e-5 at bs32 from the same random init on every client, ONE FedAvg
   round over all ranks, then ``evaluate_model`` of the aggregate on each
   client's 4,515 test rows (client1.py:379-401; reference numbers
   client1_aggregated_metrics.csv:2 / client2_aggregated_metrics.csv:2).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
With --gpus N > 1 and no torch.distributed environment, bench.py starts
``python -m torch.distributed.run --nproc-per-node N`` as a CHILD process
(before any GPU call; the parent never touches the GPU) and exits with its
status; every rank checks WORLD_SIZE == N.  Rank 0 prints ONE JSON line;
value = aggregate batches/s over all clients.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

PKG = "detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd"
BASELINE_BATCHES_PER_SEC_PER_CLIENT = 2.5  # BASELINE.md (bs16 fp32, Windows PC)
HEADLINE_METRIC = "batches/sec/client (DistilBERT seq128 bs32) + aggregated F1 after 1 FedAvg round, 1/2/4/8 MI355X"


def _args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch-size", type=int, default=32)
    ap.add_argument("--seq-len", type=int, default=128)
    ap.add_argument("--impl", default="hip", choices=["hip", "torch"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-group-dw", action="store_true", help="one launch per weight gradient (A/B)")
    ap.add_argument("--spinup-seconds", type=float, default=1.0,
                    help="busy the GPU with a plain matmul loop before the warmup steps (a GPU that was idle "
                         "runs the first ~100 ms of work measurably slower); no model state is touched")
    ap.add_argument("--step-events", action="store_true",
                    help="diagnostic: per-step GPU times from events recorded between the timed steps")
    ap.add_argument("--no-quality", action="store_true",
                    help="skip the post-timing 3-epoch + FedAvg quality protocol (kernel profiles of the step alone)")
    ap.add_argument("--quality-rows", type=int, default=None,
                    help="rows of the synthetic file the quality protocol samples 10 %% of "
                         "(default 225,745 on GPU = the Friday-DDoS file; 2,000 on CPU)")
    ap.add_argument("--quality-epochs", type=int, default=None, help="local epochs (default 3 on GPU, 1 on CPU)")
    ap.add_argument("--data-profile", default="default", choices=["default", "calibrated", "hard"],
                    help="synthetic generator setting of the quality half (data/synthetic.py PROFILES)")
    ap.add_argument("--no-defer-dw", action="store_true",
                    help="reduce each split-K weight gradient right after its GEMM instead of once per step (A/B)")
    ap.add_argument("--no-fuse-colsum", action="store_true",
                    help="separate column-sum pass for FFN lin1's bias gradient (A/B)")
    ap.add_argument("--no-fused-adam", action="store_true",
                    help="store the weight gradients and run Adam separately instead of applying it in the "
                         "all-layer weight-gradient GEMM's epilogue (A/B)")
    ap.add_argument("--padded", action="store_true",
                    help="run the blocks on all B*S positions instead of the packed real tokens (A/B)")
    ap.add_argument("--layers", type=int, default=6)
    ap.add_argument("--comm", default="torch", choices=["torch", "rccl"],
                    help="FedAvg collective: torch.distributed (RCCL) or the framework's NativeComm (RCCL)")
    ap.add_argument("--gpus-per-client", type=int, default=1,
                    help="k > 1: each federated client is k data-parallel GPUs (per-step gradient all-reduce); "
                         "--batch-size stays the per-client batch")
    ap.add_argument("--mode", default="train", choices=["train", "infer"],
                    help="infer: serving throughput of the HIP-graph forward (reference evaluate_model rate)")
    ap.add_argument("--teacher", action="store_true",
                    help="distillation step (BASELINE.json config 5): BERT-base teacher fwd + DistilBERT student")
    ap.add_argument("--lr", type=float, default=2e-5, help="Adam learning rate of the quality protocol "
                    "(reference client1.py:380: 2e-5)")
    ap.add_argument("--kd-alpha", type=float, default=0.9,
                    help="distillation loss weight of the CE term: alpha CE + (1 - alpha) T^2 KL")
    ap.add_argument("--kd-temperature", type=float, default=2.0)
    ap.add_argument("--virtual-clients", type=int, default=2,
                    help="one-GPU job: the quality protocol trains this many federated clients in turn on the "
                         "GPU (seeds 42, 43, ...) and averages them -- the reference's 2-client FedAvg round "
                         "(1: a single client, whose FedAvg is an identity)")
    ap.add_argument("--warm-start-epochs", type=int, default=0,
                    help="virtual-client quality protocol: first train the shared init this many epochs on a "
                         "separate public synthetic file (fed/runner.py warm_start) -- the analog of the "
                         "reference's pretrained DistilBERT start (client1.py:56)")
    ap.add_argument("--rounds", type=int, default=1,
                    help="FedAvg rounds of the quality protocol (BASELINE.json config 4: 3); each round every "
                         "client restarts from the previous aggregate with a fresh Adam (client1.py:375-380)")
    return ap.parse_args(argv)


# ----------------------------------------------------------------------------- launcher
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def _visible_gpus(nodes_dir: str = KFD_NODES) -> int:
    """GPUs this process may use, counted WITHOUT any GPU library: the KFD topology nodes with a
    nonzero ``gpu_id`` (CPU nodes have 0), capped by ``ROCR_VISIBLE_DEVICES`` /
    ``HIP_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES`` (an empty list hides every GPU).  The
    launcher parent must not initialise the GPU runtime before it starts the rank processes
    (torch.cuda.device_count() can fall back to hipGetDeviceCount).  0 = unknown / none."""
    n = 0
    try:
        for node in os.listdir(nodes_dir):
            try:
                with open(os.path.join(nodes_dir, node, "gpu_id")) as f:
                    n += int(f.read().strip() or 0) != 0
            except (OSError, ValueError):
                continue
    except OSError:
        return 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def _gpu_runtime_mapped() -> bool:
    """Whether this process has opened the GPU (the KFD device is mapped once HSA initialises)."""
    try:
        with open("/proc/self/maps") as f:
            return any("/dev/kfd" in ln for ln in f)
    except OSError:
        return False


def _spawn(args) -> int:
    """--gpus N > 1 without a torch.distributed environment: run N ranks as a child
    ``torch.distributed.run`` (one process per GPU, rendezvous on 127.0.0.1) and return its
    exit status.  Nothing here initialises the GPU: the GPUs are counted from sysfs, and the
    children learn (FEDDDOS_PARENT_GPU_INIT) whether the parent's address space held the GPU
    device at the moment of the spawn -- rank 0 reports it as ``parent_gpu_initialized``."""
    ngpu = _visible_gpus()
    shared = os.environ.get("FEDDDOS_BACKEND") == "gloo"  # functional runs: ranks may share a device
    if ngpu and ngpu < args.gpus and not shared:
        print(f"bench: --gpus {args.gpus} needs {args.gpus} GPUs (one rank per GPU over RCCL), "
              f"but this machine has {ngpu}; refusing to report a smaller run", file=sys.stderr, flush=True)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    env["FEDDDOS_PARENT_GPU_INIT"] = "1" if _gpu_runtime_mapped() else "0"
    return subprocess.call(cmd, env=env)


# ----------------------------------------------------------------------------- main
def main():
    args = _args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_spawn(args))

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from importlib import import_module
    comm = import_module(f"{PKG}.parallel.comm")
    fedavg = import_module(f"{PKG}.parallel.fedavg")
    models = import_module(f"{PKG}.models")
    engine = import_module(f"{PKG}.engine")
    data = import_module(f"{PKG}.data")
    runner = import_module(f"{PKG}.fed.runner")
    config = import_module(f"{PKG}.config")

    di = comm.init_distributed()
    if di.world_size != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but the process group has {di.world_size} rank(s)")
    dev = di.device
    if di.distributed and dev.type == "cuda" and di.backend != "nccl" and "FEDDDOS_BACKEND" not in os.environ:
        raise SystemExit(f"bench: GPU ranks must use RCCL (backend 'nccl'), got {di.backend!r}")
    B, S = args.batch_size, args.seq_len
    on_gpu = dev.type == "cuda"

    # ---- the client: its data split (also the throughput batches) and, later, the protocol
    q_rows = args.quality_rows or (225_745 if on_gpu else 2_000)
    q_epochs = args.quality_epochs or (3 if on_gpu else 1)
    fc = config.FedConfig(synthetic_rows=q_rows, batch_size=B, eval_batch_size=16, epochs=q_epochs, rounds=1,
                          max_len=S, impl=args.impl, gpus_per_client=args.gpus_per_client, comm=args.comm,
                          out_dir=os.path.join(os.environ.get("TMPDIR", "/tmp"), f"fedddos_bench_{os.getpid()}"),
                          plots=False, resume=False, save_checkpoints=False, heartbeat_s=0.0, verbose=False,
                          teacher="bert-base" if args.teacher else None, lr=args.lr, kd_alpha=args.kd_alpha,
                          kd_temperature=args.kd_temperature, data_profile=args.data_profile)
    client = runner.FederatedClient(fc, model_config=models.DistilBertConfig(n_layers=args.layers))
    topo = client.topo
    k = topo.gpus_per_client
    t_setup = time.perf_counter()
    client.setup()
    t_setup = time.perf_counter() - t_setup
    train = client.data.train
    loader = data.DeviceLoader(train, B, shuffle=True, device=dev, seed=topo.client_idx, drop_last=True)
    if topo.dp:
        loader = import_module(f"{PKG}.parallel.dp").DPShardLoader(loader, topo.dp_rank, k)

    # ---- the throughput model (same architecture and init; discarded after the timed window)
    cfg = models.DistilBertConfig(n_layers=args.layers)
    model = models.DDoSClassifier(config=cfg, device=dev, impl=args.impl, seed=0)
    model.group_dw = not args.no_group_dw
    model.defer_dw_reduce = not args.no_defer_dw
    model.fuse_colsum = not args.no_fuse_colsum
    ncomm = client.comm
    fedavg.broadcast_model(model, comm=ncomm)
    opt = engine.ArenaAdam(model, lr=2e-5, fuse_dw=not args.no_fused_adam)
    gsync = None
    teacher = None
    if args.teacher:
        teacher = models.BertTeacherClassifier(config=models.bert_base_config(), device=dev, impl=args.impl)
        fedavg.broadcast_model(teacher, comm=ncomm)
        teacher.eval()
    if topo.dp:
        dp = import_module(f"{PKG}.parallel.dp")
        dp.dp_seed_offset(model, topo.dp_rank)
        gsync = dp.GradSync(model, topo.dp_group, k, max_rows=B * S, ncomm=client.dp_comm)
        gsync.set_loss_scale(1.0 / k)
        fn = dp.make_dp_step_fn(model, opt, gsync, teacher, args.kd_temperature, args.kd_alpha)
    elif args.teacher:
        fn = engine.make_kd_step_fn(model, teacher, opt, args.kd_temperature, args.kd_alpha)
    else:
        fn = engine.make_step_fn(model, opt)
    model.unpad = not args.padded
    # (a data-parallel client's step is captured too when its exchange runs over the client's own
    # NativeComm -- fed/runner.py dp_comm; torch.distributed's collectives are not capturable)
    # the HIP head kernel adds each step's mean loss to this device scalar (captured into the
    # graph), so the timed loop launches nothing per step besides the graph replay itself
    dev_acc = args.impl == "hip" and on_gpu
    model.loss_acc = torch.zeros(1, device=dev) if dev_acc else None
    step = engine.GraphedTrainStep(fn, warmup=2, enabled=(not args.no_graph) and args.impl == "hip"
                                   and on_gpu and (gsync is None or gsync.capturable),
                                   bucket=getattr(model, "packed_rows", None))
    model.train()

    def batches():
        while True:
            for b in loader:
                yield b

    it = batches()

    def spinup():
        if on_gpu and args.spinup_seconds > 0:
            a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
            t_end = time.perf_counter() + args.spinup_seconds
            while time.perf_counter() < t_end:
                for _ in range(20):
                    a = (a @ a).clamp_(-1.0, 1.0)
                torch.cuda.synchronize()
            del a

    if args.mode == "infer":
        spinup()
        return _bench_infer(args, model, it, di, comm, B, S)
    # The timed batches are drawn up front; any packed-row bucket among them without a
    # captured graph yet gets one extra (untimed) training step on that batch, so no HIP
    # graph capture happens inside the timed region.  The W warmup steps run after that
    # host-side work, right before the timed region, so the GPU enters it at full clock.
    warm = [next(it) for _ in range(args.warmup)]
    n_early = min(len(warm), max(0, step.warmup) if step.enabled else 0)
    for b in warm[:n_early]:
        step(b["input_ids"], b["attention_mask"], b["labels"], b.get("n_tokens"))
    timed = [next(it) for _ in range(args.steps)]
    if step.enabled and step.bucket is not None and model.unpad:
        primed = set()
        for b in timed:
            key = step._key(b["input_ids"], b.get("n_tokens"))
            if key not in step.graphs and key not in primed and not step.failed:
                primed.add(key)
                step(b["input_ids"], b["attention_mask"], b["labels"], b.get("n_tokens"))
    if di.distributed:
        fedavg.fedavg_(model, weight=1.0 / k, comm=ncomm)
    sync = torch.cuda.synchronize if on_gpu else (lambda: None)
    # Python's cyclic GC is collected here and paused over the timed loop (host-side
    # housekeeping kept out of the timed region).
    gc.collect()
    gc.disable()
    loss_acc = torch.zeros((), device=dev)
    # All host-side preparation (graph captures, batch draws, GC) is done: bring the GPU to its
    # working clock with the spin-up loop, then run the remaining warmup steps back to back and go
    # straight into the timed loop.  (With the spin-up before the captures the idle gap let the
    # clock fall again: the first timed steps of a 20-step window ran at 1.91 / 1.70 ms against a
    # 1.57 ms steady state -- profiles/r6_step_events_window.txt.)
    sync()
    spinup()
    # the warmup steps accumulate their loss exactly like the timed loop, so the first timed
    # step does not pay the one-time load of torch's add kernel
    warm_acc = torch.zeros((), device=dev)
    for b in warm[n_early:]:
        out = step(b["input_ids"], b["attention_mask"], b["labels"], b.get("n_tokens"))
        if not dev_acc:
            warm_acc += out
    if dev_acc:
        model.loss_acc.zero_()
    sync()
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(len(timed) + 1)] if args.step_events else None
    if evs:
        evs[0].record()
    for i, b in enumerate(timed):
        out = step(b["input_ids"], b["attention_mask"], b["labels"], b.get("n_tokens"))
        if not dev_acc:
            loss_acc += out
        if evs:
            evs[i + 1].record()
    host_s = time.perf_counter() - t0  # host-side submission of the K steps (diagnostic)
    gc.enable()
    # (the window holds the K local training steps only -- the reference's 2.5 batches/s is its
    # local-epoch rate, client1_terminal_output.txt:7 -- and the FedAvg round, one per 2,541 local
    # steps in the reference protocol, is timed on its own below: fedavg_round_ms.  One round
    # inside a 20-step window would be charged at 127x its real per-step share.)
    sync()
    comm.barrier()
    sync()
    dt_rank = time.perf_counter() - t0
    if args.impl == "hip" and on_gpu and getattr(model, "fuse_ln", False):
        # a LayerNorm-fused GEMM whose row-block rendezvous timed out inside the timed window
        # produced wrong statistics: fail loudly instead of reporting its throughput
        import_module(f"{PKG}.ops.kernels").check_ln_error(dev, cfg.dim)
    per_rank_ms = [round(1000.0 * v[0] / args.steps, 4) for v in comm.all_gather_floats([dt_rank])]
    dt = comm.all_reduce_max(dt_rank)
    loss = float((model.loss_acc if dev_acc else loss_acc).sum().item()) / args.steps
    if not (loss == loss and abs(loss) < 1e6):
        raise SystemExit(f"bench: non-finite training loss {loss} -- refusing to report a throughput")
    tok = [int(b["n_tokens"]) for b in timed if b.get("n_tokens") is not None]
    real_frac = (sum(tok) / (len(tok) * B * S)) if tok else 1.0
    rows_frac = (sum(model.packed_rows(t, B, S) for t in tok) / (len(tok) * B * S)) \
        if tok and model.unpad and args.impl == "hip" else 1.0
    comm_stats = _fedavg_timing(model, di, fedavg, comm, ncomm, k, sync)
    graphs = len(getattr(step, "graphs", {}))
    graph_ok = step.graph is not None
    graph_chain = step.graph_count
    graph_err = step.failed
    fused = bool(opt.can_fuse()) and gsync is None
    del step, fn, opt, model, warm, timed, it, loader, gsync, teacher
    gc.collect()
    if on_gpu:
        torch.cuda.empty_cache()

    # ---- quality: 3 local epochs + 1 FedAvg round through the federated client (untimed)
    quality = {} if args.no_quality else _quality(client, di, comm, q_rows, q_epochs, on_gpu,
                                                  n_virtual=args.virtual_clients, n_rounds=args.rounds,
                                                  warm_epochs=args.warm_start_epochs)
    n = di.world_size
    clients = topo.num_clients
    per_client = args.steps / dt
    if di.is_main:
        default_cfg = (S == 128 and B == 32 and args.layers == 6 and not args.teacher)
        # a non-default config names its real workload: the rows are padded to S, but the packed
        # step runs on the real tokens only (CICIDS2017 text is ~80 WordPiece tokens a row)
        metric = HEADLINE_METRIC if default_cfg else (
            f"batches/sec/client (DistilBERT{'' if args.layers == 6 else f' {args.layers}-layer'} seq{S} bs{B}"
            + (f", mean {real_frac * S:.0f} real tokens/row" if real_frac < 1.0 else "")
            + (" KD from BERT-base teacher" if args.teacher else "") + ") + aggregated F1 after 1 FedAvg round")
        out = {
            "metric": metric,
            "value": round(per_client * clients, 4),
            "unit": f"batches/s (sum over clients; bs{B} x seq{S})",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * dt / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(per_client / BASELINE_BATCHES_PER_SEC_PER_CLIENT, 3),
            "dtype": "bf16" if args.impl == "hip" else "fp32",
            "data": "synthetic CICIDS2017-shaped flows rendered to text (the client's 10 % sample of a "
                    f"{q_rows:,}-row synthetic file), WordPiece seq{S}; random-init weights",
            "config": {"model": f"DistilBERT-base ({args.layers} layers) + Linear(768,2) DDoSClassifier"
                                + (" <- KD from BERT-base teacher" if args.teacher else ""),
                       "global_batch": B * clients, "seq_len": S,
                       "parallelism": f"fedavg{n} (1 client/GPU)" if k == 1 else f"fedavg{clients} x dp{k}"},
            "per_client_batches_per_sec": round(per_client, 4),
            "samples_per_sec_total": round(per_client * clients * B, 2),
            "tokens_per_sec_total": round(per_client * clients * B * S, 1),
            "vs_baseline_basis": "per-client batches/s / 2.5 (reference bs16 fp32 per-client rate)",
            "per_rank_ms_per_step": per_rank_ms,
            "backend": di.backend,
            "real_token_fraction": round(real_frac, 4),
            "mean_real_tokens_per_row": round(real_frac * S, 1),
            "packed_row_fraction": round(rows_frac, 4),
            "impl": args.impl,
            "comm": args.comm,
            "spinup_s": args.spinup_seconds,
            "setup_s": round(t_setup, 2),
            "hip_graph": graph_ok,
            "hip_graph_chain": graph_chain,
            "hip_graphs": graphs,
            "unpadded": bool(rows_frac < 1.0),
            "fused_adam": fused,
            "graph_error": graph_err,
            "host_submit_ms": round(1000.0 * host_s, 2),
            **({"parent_gpu_initialized": os.environ["FEDDDOS_PARENT_GPU_INIT"] == "1"}
               if "FEDDDOS_PARENT_GPU_INIT" in os.environ else {}),
            **({"step_ms": [round(evs[i].elapsed_time(evs[i + 1]), 3) for i in range(len(evs) - 1)]} if evs else {}),
            "mean_loss": round(loss, 5),
            "timed_region": "K local training steps (forward + backward + Adam); the FedAvg round is timed "
                            "separately (fedavg_round_ms)",
            **comm_stats,
            # the round charged at the reference protocol's rate: one FedAvg per 3 epochs x 847 steps
            **({"ref_steps_per_round": REF_STEPS_PER_ROUND,
                "ms_per_step_incl_round": round(1000.0 * dt / args.steps
                                                + comm_stats["fedavg_round_ms"] / REF_STEPS_PER_ROUND, 4)}
               if comm_stats.get("fedavg_round_ms") is not None else {}),
            **quality,
        }
        print(json.dumps(out), flush=True)
    comm.shutdown()


REF_STEPS_PER_ROUND = 3 * 847  # local steps per FedAvg round in the reference (client1_terminal_output.txt:7-11)


def _fedavg_timing(model, di, fedavg, comm, ncomm, k, sync):
    """FedAvg round time (all-reduce of the 265 MB fp32 arena + fused scale/cast) and the raw
    all-reduce's bus bandwidth, 2(N-1)/N x bytes / t (untimed diagnostics, max over ranks)."""
    if not di.distributed:
        return {"fedavg_round_ms": None, "fedavg_ms": None, "allreduce_ms": None, "allreduce_busbw_GBps": None}
    A = model.arena.master
    nbytes = A.numel() * A.element_size()
    n = di.world_size
    fed, raw = [], []
    scratch = torch.empty_like(A)
    for _ in range(3):
        sync()
        comm.barrier()
        t = time.perf_counter()
        fedavg.fedavg_(model, weight=1.0 / k, comm=ncomm)
        sync()
        fed.append(time.perf_counter() - t)
    import torch.distributed as dist
    for _ in range(3):
        scratch.copy_(A)
        sync()
        comm.barrier()
        t = time.perf_counter()
        if ncomm is not None and scratch.is_cuda:
            ncomm.all_reduce_(scratch, "sum", wait=False)  # (timed to the sync below)
        else:
            dist.all_reduce(scratch)
        sync()
        raw.append(time.perf_counter() - t)
    del scratch
    f = comm.all_reduce_max(min(fed))
    f0 = comm.all_reduce_max(fed[0])  # the first round after the timed steps (what a real round sees)
    r = comm.all_reduce_max(min(raw))
    fm = comm.all_reduce_max(float(np.median(fed)))
    return {"fedavg_round_ms": round(1e3 * f0, 3), "fedavg_ms": round(1e3 * f, 3),
            "fedavg_round_ms_median": round(1e3 * fm, 3), "fedavg_rounds_timed": len(fed),
            "allreduce_ms": round(1e3 * r, 3),
            "allreduce_bytes": nbytes,
            "allreduce_busbw_GBps": round(2.0 * (n - 1) / n * nbytes / r / 1e9, 2)}


def _quality_virtual(client, rows, epochs, on_gpu, n_virtual, n_rounds=1, warm_epochs=0):
    """1-GPU job: the reference's 2-client round with both clients trained one after the other on
    this GPU (fed/runner.py run_virtual_clients): seeds 42 / 43, the same init, 3 local epochs each,
    the FedAvg sum + scale_cast, each client's test split evaluated on its local model and on the
    aggregate (client1_local_metrics.csv / client1_aggregated_metrics.csv)."""
    from importlib import import_module
    runner = import_module(f"{PKG}.fed.runner")
    t0 = time.perf_counter()
    warm = None
    if warm_epochs > 0:
        warm = runner.warm_start(client, warm_epochs, rows=rows)
        print(f"[quality] warm start: {warm_epochs} epoch(s) on a public synthetic file, public test "
              f"{warm['public_test']['accuracy']:.3f} %", file=sys.stderr, flush=True)
    res = runner.run_virtual_clients(client, n_virtual, rounds=n_rounds,
                                     progress=lambda m: print(f"[quality] {m}", file=sys.stderr, flush=True))
    if on_gpu:
        torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    (tn, fp), (fn, tp) = res["aggregated_confusion"]
    prec = tp / (tp + fp) if tp + fp else 0.0
    rec_ = tp / (tp + fn) if tp + fn else 0.0
    f1 = 2 * prec * rec_ / (prec + rec_) if prec + rec_ else 0.0
    total = tp + fp + fn + tn
    cl = res["clients"]
    cl1 = res["rounds"][0]["clients"]  # (the teachers are fine-tuned in each client's first round)
    return {"aggregated_f1": round(f1, 5),
            "aggregated_accuracy_pct": round(100.0 * (tp + tn) / max(total, 1), 3),
            "aggregated_confusion": [[int(tn), int(fp)], [int(fn), int(tp)]],
            "min_client_aggregated_accuracy_pct": round(min(c["aggregated_test"]["accuracy"] for c in cl), 3),
            "min_client_aggregated_f1": round(min(c["aggregated_test"]["f1"] for c in cl), 5),
            "mean_client_local_accuracy_pct": round(float(np.mean([c["local_test"]["accuracy"] for c in cl])), 3),
            "mean_client_local_f1": round(float(np.mean([c["local_test"]["f1"] for c in cl])), 5),
            "quality_virtual_clients": n_virtual,
            "quality_clients": n_virtual,
            "per_client": [{"client": c["client"], "seed": client.cfg.client_seed(c["client"] - 1),
                            "train_rows": c["train_rows"], "test_rows": c["test_rows"],
                            "local_accuracy_pct": round(c["local_test"]["accuracy"], 3),
                            "local_f1": round(c["local_test"]["f1"], 5),
                            "aggregated_accuracy_pct": round(c["aggregated_test"]["accuracy"], 3),
                            "aggregated_f1": round(c["aggregated_test"]["f1"], 5),
                            "aggregated_confusion": c["aggregated_test"]["confusion_matrix"],
                            "rel_l2_local_to_aggregate": float(f"{c['rel_l2_local_to_aggregate']:.4e}"),
                            "epoch_losses": [round(x, 5) for x in c["train"]["epoch_losses"]],
                            "train_steps": c["train"]["steps"]} for c in cl],
            "eval_rows": int(total), "eval_rows_per_client": int(total) // max(len(cl), 1),
            "train_rows_per_client": cl[0]["train_rows"], "fedavg_rounds": n_rounds, "local_epochs": epochs,
            **({"per_round": [_round_summary(h) for h in res["rounds"]]} if n_rounds > 1 or warm else {}),
            **({"warm_start": {"epochs": warm_epochs, "public_rows": warm["rows"], "public_seed": warm["seed"],
                               "public_train_rows": warm["train_rows"],
                               "public_test_accuracy_pct": round(warm["public_test"]["accuracy"], 3),
                               "public_test_f1": round(warm["public_test"]["f1"], 5)}} if warm else {}),
            "quality_file_rows": rows, "quality_fedavg_ms": round(res["fedavg_ms"], 3),
            "quality_train_batches_per_sec": round(float(np.mean([c["train"]["batches_per_sec"] for c in cl])), 2),
            "quality_wall_s": round(wall, 2), "quality_lr": client.cfg.lr,
            **({"kd_alpha": client.cfg.kd_alpha, "kd_temperature": client.cfg.kd_temperature,
                "teacher_test_accuracy_pct": round(float(np.mean([c["teacher_test"]["accuracy"] for c in cl1])), 3),
                "teacher_test_f1": round(float(np.mean([c["teacher_test"]["f1"] for c in cl1])), 5),
                "per_client_teacher": [{"client": c["client"], "accuracy_pct": round(c["teacher_test"]["accuracy"], 3),
                                        "f1": round(c["teacher_test"]["f1"], 5),
                                        "confusion": c["teacher_test"]["confusion_matrix"]} for c in cl1]}
               if client.teacher is not None else {})}


def _acc_f1(cm):
    (tn, fp), (fn, tp) = cm
    prec = tp / (tp + fp) if tp + fp else 0.0
    rec_ = tp / (tp + fn) if tp + fn else 0.0
    f1 = 2 * prec * rec_ / (prec + rec_) if prec + rec_ else 0.0
    return 100.0 * (tp + tn) / max(tp + tn + fp + fn, 1), f1


def _round_summary(h):
    """One FedAvg round of the virtual-client protocol: pooled and per-client local / aggregated
    accuracy, F1 and confusion (the reference's clientN_{local,aggregated}_metrics.csv, per round)."""
    acc, f1 = _acc_f1(h["aggregated_confusion"])
    lacc, lf1 = _acc_f1(h["local_confusion"])
    cl = h["clients"]
    return {"round": h["round"], "aggregated_accuracy_pct": round(acc, 3), "aggregated_f1": round(f1, 5),
            "aggregated_confusion": h["aggregated_confusion"], "local_accuracy_pct": round(lacc, 3),
            "local_f1": round(lf1, 5), "local_confusion": h["local_confusion"],
            "min_client_aggregated_accuracy_pct": round(min(c["aggregated_test"]["accuracy"] for c in cl), 3),
            "min_client_aggregated_f1": round(min(c["aggregated_test"]["f1"] for c in cl), 5),
            "fedavg_ms": round(h["fedavg_ms"], 3),
            "clients": [{"client": c["client"], "local_accuracy_pct": round(c["local_test"]["accuracy"], 3),
                         "local_f1": round(c["local_test"]["f1"], 5),
                         "local_confusion": c["local_test"]["confusion_matrix"],
                         "aggregated_accuracy_pct": round(c["aggregated_test"]["accuracy"], 3),
                         "aggregated_f1": round(c["aggregated_test"]["f1"], 5),
                         "aggregated_confusion": c["aggregated_test"]["confusion_matrix"],
                         "epoch_losses": [round(x, 5) for x in c["train"]["epoch_losses"]],
                         "rel_l2_local_to_aggregate": float(f"{c['rel_l2_local_to_aggregate']:.4e}"),
                         **({"teacher_accuracy_pct": round(c["teacher_test"]["accuracy"], 3),
                             "teacher_f1": round(c["teacher_test"]["f1"], 5)} if "teacher_test" in c else {})}
                        for c in cl]}


def _quality(client, di, comm, rows, epochs, on_gpu, n_virtual=1, n_rounds=1, warm_epochs=0):
    """Run round 1 of the federated client (fed/runner.py run_round: local train -> local eval
    -> FedAvg -> aggregated eval) and pool the aggregated test confusion matrices of all clients.
    n_virtual > 1 (a one-process job): that many clients trained in turn on this device instead."""
    if (n_virtual > 1 or n_rounds > 1 or warm_epochs > 0) and not di.distributed:
        return _quality_virtual(client, rows, epochs, on_gpu, n_virtual, n_rounds, warm_epochs)
    t0 = time.perf_counter()
    client.cfg.rounds = n_rounds
    per_round = []
    for r in range(n_rounds):
        rec = client.run_round(r)
        if n_rounds > 1:
            cm = rec["aggregated_test"]["confusion_matrix"]
            w = 1.0 if client.topo.dp_rank == 0 else 0.0  # data-parallel replicas share one client's split
            v = [w * float(x) for row in cm for x in row] if len(cm) == 2 else [0.0] * 4
            pooled = [sum(x[i] for x in comm.all_gather_floats(v)) for i in range(4)]
            acc, f1 = _acc_f1([[pooled[0], pooled[1]], [pooled[2], pooled[3]]])
            per_round.append({"round": r + 1, "aggregated_accuracy_pct": round(acc, 3),
                              "aggregated_f1": round(f1, 5)})
    if on_gpu:
        torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    agg, loc = rec["aggregated_test"], rec["local_test"]
    (tn, fp), (fn, tp) = agg["confusion_matrix"] if len(agg["confusion_matrix"]) == 2 else ((0, 0), (0, 0))
    writer = 1.0 if client.topo.dp_rank == 0 else 0.0  # data-parallel replicas share one client's split
    vec = [writer * v for v in (tp, fp, fn, tn, agg["accuracy"], agg["f1"], loc["accuracy"], loc["f1"])]
    allv = [v for v in comm.all_gather_floats(vec + [writer]) if v[-1] > 0]
    tp, fp, fn, tn = (sum(v[i] for v in allv) for i in range(4))
    prec = tp / (tp + fp) if tp + fp else 0.0
    rec_ = tp / (tp + fn) if tp + fn else 0.0
    f1 = 2 * prec * rec_ / (prec + rec_) if prec + rec_ else 0.0
    total = tp + fp + fn + tn
    tr = rec["train"]
    return {"aggregated_f1": round(f1, 5),
            "aggregated_accuracy_pct": round(100.0 * (tp + tn) / max(total, 1), 3),
            "aggregated_confusion": [[int(tn), int(fp)], [int(fn), int(tp)]],
            "min_client_aggregated_accuracy_pct": round(min(v[4] for v in allv), 3),
            "min_client_aggregated_f1": round(min(v[5] for v in allv), 5),
            "mean_client_local_accuracy_pct": round(float(np.mean([v[6] for v in allv])), 3),
            "mean_client_local_f1": round(float(np.mean([v[7] for v in allv])), 5),
            "eval_rows": int(total), "eval_rows_per_client": int(total) // max(len(allv), 1),
            "train_rows_per_client": len(client.data.train), "quality_clients": len(allv),
            "fedavg_rounds": n_rounds, "local_epochs": epochs, "quality_file_rows": rows,
            **({"per_round": per_round} if per_round else {}),
            "quality_epoch_losses": [round(x, 5) for x in tr["epoch_losses"]],
            "quality_train_steps": tr["steps"], "quality_train_batches_per_sec": round(tr["batches_per_sec"], 2),
            "quality_fedavg_ms": round(rec["fedavg_ms"], 3), "quality_wall_s": round(wall, 2),
            "quality_lr": client.cfg.lr,
            **({"kd_alpha": client.cfg.kd_alpha, "kd_temperature": client.cfg.kd_temperature}
               if client.teacher is not None else {}),
            **({"teacher_test_accuracy_pct": round(rec["teacher_test"]["accuracy"], 3),
                "teacher_test_f1": round(rec["teacher_test"]["f1"], 5)} if "teacher_test" in rec else {})}


def _bench_infer(args, model, it, di, comm, B, S):
    """Inference batches/s (no grad, HIP-graph forward, probabilities + labels on device).
    Reference: evaluate_model at 8.87-14.0 batches/s of 16 rows (client1_terminal_output.txt:16,21)."""
    from importlib import import_module
    engine = import_module(f"{PKG}.engine")
    fwd = engine.GraphedForward(model, enabled=not args.no_graph)
    model.eval()
    dev = model.device
    batches = [next(it) for _ in range(args.warmup + args.steps)]
    probs = torch.empty(args.steps, B, device=dev)
    # warm every (shape, bucket) graph before timing, with the same post-processing as the
    # timed loop (so no kernel is launched for the first time inside the timed region)
    for b in batches:
        logits = fwd(b["input_ids"], b["attention_mask"], b.get("n_tokens"))
        probs[0] = torch.softmax(logits.float(), dim=1)[:, 1]
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    sync()
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    for i, b in enumerate(batches[args.warmup:]):
        logits = fwd(b["input_ids"], b["attention_mask"], b.get("n_tokens"))
        probs[i] = torch.softmax(logits.float(), dim=1)[:, 1]
    sync()
    comm.barrier()
    sync()
    dt = comm.all_reduce_max(time.perf_counter() - t0)
    n = di.world_size
    per = args.steps / dt
    if di.is_main:
        print(json.dumps({
            "metric": f"inference batches/sec/GPU (DistilBERT DDoSClassifier seq{S} bs{B})", "value": round(per * n, 3),
            "unit": f"batches/s (sum over GPUs; bs{B} x seq{S})", "n_gpus": n, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1000.0 * dt / args.steps, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": round(per * B / (14.0 * 16), 3),
            "vs_baseline_basis": "rows/s / 224 (reference evaluate_model best: 14.0 batches/s x 16 rows)",
            "dtype": "bf16" if args.impl == "hip" else "fp32", "data": "synthetic CICIDS2017-shaped flows; random-init",
            "config": {"model": "DistilBERT-base + Linear(768,2)", "global_batch": B * n, "seq_len": S,
                       "parallelism": f"replicated x{n}"},
            "rows_per_sec_total": round(per * n * B, 1), "hip_graphs": len(fwd.graphs), "graph_error": fwd.failed}),
            flush=True)
    comm.shutdown()


if __name__ == "__main__":
    main()
