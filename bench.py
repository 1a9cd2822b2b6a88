#!/usr/bin/env python3
"""Headline benchmark: local federated-client training throughput.

Metric (BASELINE.json): batches/sec/client of DistilBERT-base DDoSClassifier
training at seq_len 128, batch 32, bf16 compute, on synthetic CICIDS2017-shaped
flows rendered to text (random-init weights), one client per GPU.

A "step" is the full reference step (client1.py:102-112): forward, CE loss,
backward, Adam update -- here the fused HIP kernels replayed as a HIP graph.
For N > 1 every rank is an independent federated client and the timed region
also ends with one FedAvg round (RCCL all-reduce of the 66.4 M fp32 masters),
i.e. communication is charged once per K steps (the reference averages once per
3 epochs = 1,270 steps at bs32, so this over-charges it).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
N > 1 is launched by torch.distributed.run (one process per GPU, RCCL).
Rank 0 prints ONE JSON line; value = aggregate batches/s over all clients.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

import numpy as np
import torch

PKG = "detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd"
BASELINE_BATCHES_PER_SEC_PER_CLIENT = 2.5  # BASELINE.md (bs16 fp32, Windows PC)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch-size", type=int, default=32)
    ap.add_argument("--seq-len", type=int, default=128)
    ap.add_argument("--impl", default="hip", choices=["hip", "torch"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-group-dw", action="store_true", help="one launch per weight gradient (A/B)")
    ap.add_argument("--overlap-transpose", action="store_true", help="W^T copies on a side stream (A/B; slower)")
    ap.add_argument("--spinup-seconds", type=float, default=1.0,
                    help="busy the GPU with a plain matmul loop before the warmup steps (a GPU that was idle "
                         "runs the first ~100 ms of work measurably slower); no model state is touched")
    ap.add_argument("--step-events", action="store_true",
                    help="diagnostic: per-step GPU times from events recorded between the timed steps")
    ap.add_argument("--no-quality", action="store_true",
                    help="skip the post-timing aggregated-F1 evaluation (kernel profiles of the step alone)")
    ap.add_argument("--no-defer-dw", action="store_true",
                    help="reduce each split-K weight gradient right after its GEMM instead of once per step (A/B)")
    ap.add_argument("--no-fuse-colsum", action="store_true",
                    help="separate column-sum pass for FFN lin1's bias gradient (A/B)")
    ap.add_argument("--fused-adam", action="store_true",
                    help="apply Adam inside the weight-gradient GEMM epilogues (A/B; measured no faster)")
    ap.add_argument("--padded", action="store_true",
                    help="run the blocks on all B*S positions instead of the packed real tokens (A/B)")
    ap.add_argument("--wgrad-stream", action="store_true",
                    help="run the backward's weight-gradient work on a side stream (A/B; measured slower)")
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
    args = ap.parse_args()

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from importlib import import_module
    comm = import_module(f"{PKG}.parallel.comm")
    fedavg = import_module(f"{PKG}.parallel.fedavg")
    models = import_module(f"{PKG}.models")
    engine = import_module(f"{PKG}.engine")
    data = import_module(f"{PKG}.data")

    di = comm.init_distributed()
    dev = di.device
    dp = import_module(f"{PKG}.parallel.dp")
    topo = dp.make_topology(args.gpus_per_client)
    client = topo.client_idx
    B, S = args.batch_size, args.seq_len
    n_batches = args.warmup + args.steps
    # Synthetic CICIDS2017 rows -> the reference's text template -> WordPiece ids.
    df = data.generate_cicids2017(max(n_batches * B * 2, 4096), seed=client)
    cd = data.build_client_data(df, client, data_fraction=1.0, max_len=S)
    train = cd.train
    loader = data.DeviceLoader(train, B, shuffle=True, device=dev, seed=client, drop_last=True)
    if topo.dp:
        loader = dp.DPShardLoader(loader, topo.dp_rank, topo.gpus_per_client)

    cfg = models.DistilBertConfig(n_layers=args.layers)
    model = models.DDoSClassifier(config=cfg, device=dev, impl=args.impl, seed=0)
    model.wgrad_stream = args.wgrad_stream
    model.group_dw = not args.no_group_dw
    model.defer_dw_reduce = not args.no_defer_dw
    model.fuse_colsum = not args.no_fuse_colsum
    ncomm = None
    if args.comm == "rccl" and dev.type == "cuda":
        ncomm = import_module(f"{PKG}.parallel.rccl").NativeComm()
    fedavg.broadcast_model(model, comm=ncomm)
    opt = engine.ArenaAdam(model, lr=2e-5, fuse_dw=args.fused_adam)
    gsync = None
    if topo.dp:
        teacher = None
        if args.teacher:
            teacher = models.BertTeacherClassifier(config=models.bert_base_config(), device=dev, impl=args.impl)
            fedavg.broadcast_model(teacher, comm=ncomm)
            teacher.eval()
        dp.dp_seed_offset(model, topo.dp_rank)
        gsync = dp.GradSync(model, topo.dp_group, topo.gpus_per_client, max_rows=B * S)
        gsync.set_loss_scale(1.0 / topo.gpus_per_client)
        fn = dp.make_dp_step_fn(model, opt, gsync, teacher, 2.0, 0.5)
    elif args.teacher:
        teacher = models.BertTeacherClassifier(config=models.bert_base_config(), device=dev, impl=args.impl)
        fedavg.broadcast_model(teacher, comm=ncomm)
        teacher.eval()
        fn = engine.make_kd_step_fn(model, teacher, opt, 2.0, 0.5)
    else:
        fn = engine.make_step_fn(model, opt)
    model.unpad = not args.padded
    model.overlap_transpose = args.overlap_transpose
    step = engine.GraphedTrainStep(fn, warmup=2, enabled=(not args.no_graph) and args.impl == "hip"
                                   and dev.type == "cuda" and gsync is None,
                                   bucket=getattr(model, "packed_rows", None))
    model.train()

    def batches():
        while True:
            for b in loader:
                yield b

    it = batches()
    if dev.type == "cuda" and args.spinup_seconds > 0:
        a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
        t_end = time.perf_counter() + args.spinup_seconds
        while time.perf_counter() < t_end:
            for _ in range(20):
                a = (a @ a).clamp_(-1.0, 1.0)
            torch.cuda.synchronize()
        del a
    if args.mode == "infer":
        return _bench_infer(args, model, it, di, comm, B, S)
    # The timed batches are drawn up front; any packed-row bucket among them without a
    # captured graph yet gets one extra (untimed) training step on that batch, so no HIP
    # graph capture happens inside the timed region.  The W warmup steps run after that
    # host-side work, right before the timed region, so the GPU enters it at full clock
    # (drawing the batches first left it idle for a few ms: ~9 ms more per timed run).
    # (The first warmup steps run before the draw: the graph wrapper's eager calls, so the
    # priming below captures.)
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
    # the warmup steps accumulate their loss exactly like the timed loop, so the first timed
    # step does not pay the one-time load of torch's add kernel (~13 ms on a fresh process)
    warm_acc = torch.zeros((), device=dev)
    for b in warm[n_early:]:
        warm_acc += step(b["input_ids"], b["attention_mask"], b["labels"], b.get("n_tokens"))
    k = topo.gpus_per_client
    if args.gpus > 1 or di.distributed:
        fedavg.fedavg_(model, weight=1.0 / k, comm=ncomm)
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    # Python's cyclic GC is collected here and paused over the timed loop (host-side
    # housekeeping kept out of the timed region; the host submits 50 steps in ~3 ms).
    gc.collect()
    gc.disable()
    loss_acc = torch.zeros((), device=dev)
    sync()
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(len(timed) + 1)] if args.step_events else None
    if evs:
        evs[0].record()
    for i, b in enumerate(timed):
        loss_acc += step(b["input_ids"], b["attention_mask"], b["labels"], b.get("n_tokens"))
        if evs:
            evs[i + 1].record()
    host_s = time.perf_counter() - t0  # host-side submission of the K steps (diagnostic)
    gc.enable()
    if di.distributed:
        fedavg.fedavg_(model, weight=1.0 / k, comm=ncomm)
    sync()
    comm.barrier()
    sync()
    dt = time.perf_counter() - t0
    dt = comm.all_reduce_max(dt)
    loss = float(loss_acc.item()) / args.steps
    # Second half of the metric: the FedAvg-aggregated model (the all-reduce that closes the
    # timed region) scored on every client's held-out test split -- counts summed over
    # clients, one F1 (untimed; the reference's evaluate_model after aggregation,
    # client1.py:118-150 / 330-340).
    quality = {} if args.no_quality else _aggregated_quality(model, cd.test, dev, topo, engine, data, di)
    if not (loss == loss and abs(loss) < 1e6):
        raise SystemExit(f"bench: non-finite training loss {loss} -- refusing to report a throughput")
    n = di.world_size
    clients = topo.num_clients
    per_client = args.steps / dt
    if di.is_main:
        out = {
            "metric": "batches/sec/client (DistilBERT seq128 bs32) + aggregated F1 after 1 FedAvg round, 1/2/4/8 MI355X",
            "value": round(per_client * clients, 4),
            "unit": "batches/s (sum over clients; bs32 x seq128)",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * dt / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(per_client / BASELINE_BATCHES_PER_SEC_PER_CLIENT, 3),
            "dtype": "bf16" if args.impl == "hip" else "fp32",
            "data": "synthetic CICIDS2017-shaped flows rendered to text, WordPiece seq128; random-init weights",
            "config": {"model": f"DistilBERT-base ({args.layers} layers) + Linear(768,2) DDoSClassifier"
                                + (" <- KD from BERT-base teacher" if args.teacher else ""),
                       "global_batch": B * clients, "seq_len": S,
                       "parallelism": f"fedavg{n} (1 client/GPU)" if k == 1 else f"fedavg{clients} x dp{k}"},
            "per_client_batches_per_sec": round(per_client, 4),
            "samples_per_sec_total": round(per_client * clients * B, 2),
            "tokens_per_sec_total": round(per_client * clients * B * S, 1),
            "vs_baseline_basis": "per-client batches/s / 2.5 (reference bs16 fp32 per-client rate)",
            "impl": args.impl,
            "comm": args.comm,
            "spinup_s": args.spinup_seconds,
            "hip_graph": step.graph is not None,
            "hip_graphs": len(getattr(step, "graphs", {})),
            "unpadded": bool(getattr(model, "unpad", False)) and args.impl == "hip",
            "fused_adam": bool(opt.can_fuse()) and gsync is None,
            "graph_error": step.failed,
            "host_submit_ms": round(1000.0 * host_s, 2),
            **({"step_ms": [round(evs[i].elapsed_time(evs[i + 1]), 3) for i in range(len(timed))]} if evs else {}),
            "mean_loss": round(loss, 5),
            **quality,
        }
        print(json.dumps(out), flush=True)
    comm.shutdown()


def _aggregated_quality(model, test, dev, topo, engine, data, di):
    """Accuracy / F1 of the aggregated model over all clients' test rows (one replica per client)."""
    loader = data.DeviceLoader(test, 256, shuffle=False, device=dev, drop_last=False)
    res = engine.evaluate_model(model, loader)
    lab = np.asarray(res[6], dtype=np.int64)
    pred = (np.asarray(res[7]) > 0.5).astype(np.int64)
    c = torch.tensor([int(((pred == 1) & (lab == 1)).sum()), int(((pred == 1) & (lab == 0)).sum()),
                      int(((pred == 0) & (lab == 1)).sum()), int(((pred == 0) & (lab == 0)).sum())],
                     dtype=torch.float64, device=dev)
    if topo.dp_rank != 0:
        c.zero_()  # data-parallel replicas hold the same client's split
    if di.distributed:
        torch.distributed.all_reduce(c)
    tp, fp, fn, tn = c.tolist()
    prec = tp / (tp + fp) if tp + fp else 0.0
    rec = tp / (tp + fn) if tp + fn else 0.0
    f1 = 2 * prec * rec / (prec + rec) if prec + rec else 0.0
    return {"aggregated_f1": round(f1, 5), "aggregated_accuracy_pct": round(100.0 * (tp + tn) / max(tp + fp + fn + tn, 1), 3),
            "eval_rows": int(tp + fp + fn + tn), "fedavg_rounds": 1 if di.distributed else 0}


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
