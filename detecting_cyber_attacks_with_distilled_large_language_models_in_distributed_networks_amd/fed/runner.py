"""Federated round orchestration: one process per GPU = one client.

Reference flow per client (client1.py:353-411) + server (server.py:116-137):
  preprocess -> split 60/20/20 -> train 3 epochs -> eval val/test -> save CSV +
  clientN_model.pth -> upload (TCP, gzip) -> server averages -> download ->
  eval val/test of the aggregate -> CSV + plots -> save clientN_model.pth.

Here the upload/average/download triple is ``fedavg_`` (one RCCL all-reduce of
the fp32 arena, ``parallel/fedavg.py``) and the server's duties (writing
``ddos_distilbert_model.pth``, the cross-client report) fall to rank 0.  Extras
over the reference: R rounds in-process, resume from the round sidecar,
sample-weighted FedAvg, seeded partial participation, fault injection, a
cross-client JSON report gathered with an all-gather, and clients that span
``gpus_per_client`` data-parallel GPUs (parallel/dp.py; replica 0 of each
client does the client's file output).
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, List, Optional

import torch

from ..config import FedConfig
from ..data import DeviceLoader, WordPieceTokenizer, build_client_data, generate_cicids2017
from ..engine import ArenaAdam, evaluate_model, train_model
from ..models import DDoSClassifier, DistilBertConfig
from ..parallel import comm, health
from ..parallel.dp import DPShardLoader, GradSync, dp_seed_offset, make_topology
from ..parallel.fedavg import broadcast_model, fedavg_
from ..utils import checkpoint as ck
from ..utils import faults
from ..utils.logging import TagLogger
from ..utils.metrics import save_metrics
from ..utils.timers import PhaseTimer


def _metrics_record(m) -> Dict:
    return {"accuracy": float(m[0]), "loss": float(m[1]), "precision": float(m[2]), "recall": float(m[3]),
            "f1": float(m[4]), "confusion_matrix": [[int(x) for x in row] for row in m[5]]}


class FederatedClient:
    def __init__(self, cfg: FedConfig, frame=None, model_config: Optional[DistilBertConfig] = None):
        self.cfg = cfg
        self.di = comm.init_distributed(timeout_s=cfg.timeout_s)
        self.topo = make_topology(cfg.gpus_per_client)
        self.idx = self.topo.client_idx              # 0-based client index
        self.client_id = self.idx + 1                # reference naming: Client 1, Client 2, ...
        self.num_clients = cfg.num_clients or self.topo.num_clients
        self.writer = self.topo.dp_rank == 0         # replica 0 writes the client's files
        os.makedirs(cfg.out_dir, exist_ok=True)
        sfx = "" if self.writer else f"_replica{self.topo.dp_rank}"
        self.log = TagLogger.for_client(self.client_id, enabled=cfg.verbose and self.writer,
                                        jsonl_path=os.path.join(cfg.out_dir, f"client{self.client_id}{sfx}_log.jsonl"))
        self.timer = PhaseTimer()
        self.device = self.di.device
        self.frame = frame
        self.model_config = model_config or DistilBertConfig()

    # ------------------------------------------------------------------ setup
    def setup(self):
        cfg, log = self.cfg, self.log
        log.phase("Starting client")
        with self.timer("preprocess"):
            if self.frame is None:
                if cfg.csv_path:
                    import pandas as pd
                    self.frame = pd.read_csv(cfg.csv_path)
                else:
                    # Same seeded synthetic file on every client (they sample it independently).
                    self.frame = generate_cicids2017(cfg.synthetic_rows, seed=0, profile=cfg.data_profile)
            self.tokenizer = WordPieceTokenizer.from_pretrained(cfg.model_path)
            self.data = build_client_data(self.frame, self.idx, cfg.data_fraction, cfg.base_seed, cfg.max_len,
                                          self.tokenizer, cfg.partition, self.num_clients, log=log)
        dev = self.device
        self.train_loader = DeviceLoader(self.data.train, cfg.batch_size, shuffle=True, device=dev,
                                         seed=cfg.client_seed(self.idx))
        if self.topo.dp:
            self.train_loader = DPShardLoader(self.train_loader, self.topo.dp_rank, self.topo.gpus_per_client)
        self.val_loader = DeviceLoader(self.data.val, cfg.eval_batch_size, device=dev)
        self.test_loader = DeviceLoader(self.data.test, cfg.eval_batch_size, device=dev)
        mc = self.model_config
        mc.dropout, mc.attention_dropout = cfg.hidden_dropout, cfg.attention_dropout
        self.model = DDoSClassifier(cfg.model_path, config=mc, device=dev, impl=cfg.impl, seed=0,
                                    head_dropout=cfg.head_dropout)
        self.comm = None
        if cfg.comm == "rccl" and dev.type == "cuda":
            from ..parallel.rccl import NativeComm
            self.comm = NativeComm()
            log.info(f"native RCCL communicator: {self.comm.world_size} ranks")
        # Identical start for every client: rank 0's weights win.
        broadcast_model(self.model, comm=self.comm)
        self.grad_sync = None
        self.dp_comm = None
        if self.topo.dp:
            dp_seed_offset(self.model, self.topo.dp_rank)
            # opt-in (FEDDDOS_DP_NATIVE=1) until the graph-captured exchange has run on >= 2 GPUs
            # (ADVICE r3); the default is torch.distributed's eager async all-reduces
            if dev.type == "cuda" and self.di.backend == "nccl" and os.environ.get("FEDDDOS_DP_NATIVE", "0") == "1":
                # the client's replicas exchange over a framework RCCL communicator of their own
                # group: stream-ordered collectives, so the data-parallel step is graph-captured
                from ..parallel.rccl import NativeComm
                self.dp_comm = NativeComm(group=self.topo.dp_group)
            self.grad_sync = GradSync(self.model, self.topo.dp_group, self.topo.gpus_per_client,
                                      max_rows=cfg.batch_size * cfg.max_len, ncomm=self.dp_comm)
            log.info(f"data-parallel client: replica {self.topo.dp_rank + 1}/{self.topo.gpus_per_client}")
        self.teacher = None
        if cfg.teacher:
            from ..models.bert import BertTeacherClassifier, bert_base_config
            self.teacher = BertTeacherClassifier(cfg.extra.get("teacher_path"), config=bert_base_config(),
                                                 device=dev, impl=cfg.impl)
            broadcast_model(self.teacher, comm=self.comm)
        self.teacher_sync = None
        if self.teacher is not None and self.topo.dp:
            # the teacher fine-tune is data-parallel too, so every replica distils from the same teacher
            dp_seed_offset(self.teacher, self.topo.dp_rank)
            self.teacher_sync = GradSync(self.teacher, self.topo.dp_group, self.topo.gpus_per_client,
                                         max_rows=cfg.batch_size * cfg.max_len, ncomm=self.dp_comm)
        self.start_round = 0
        self.history: List[Dict] = []
        if cfg.resume:
            self._resume()
        self.health = None
        if self.di.distributed and cfg.heartbeat_s > 0 and cfg.transport != "tcp":
            self.health = health.start(cfg.heartbeat_s, cfg.heartbeat_stale_s, cfg.timeout_s)
        restarts = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
        if restarts:
            log.info(f"elastic restart #{restarts}: resuming at round {self.start_round + 1}")
        log.info(f"data: {len(self.data.train)} train / {len(self.data.val)} val / {len(self.data.test)} test rows "
                 f"(sampled {self.data.n_rows}), impl={self.model.impl}, device={dev}")
        return self

    def _resume(self):
        """Pick ONE resume round for the whole world and start every client from that round's
        aggregate.

        The source of truth is the round tag of ``ddos_distilbert_model.pth``, which rank 0
        writes right after FedAvg and before any client records the round in its fed_state.
        Rank 0 can tag round r+1 only after every client has finished round r, so after a crash
        the tag is the last round whose aggregate exists, whatever each client's own sidecar
        says.  Rank 0 -- the rank that loads and broadcasts the aggregate -- decides, and its
        round is broadcast, so a rank that cannot see the file (a per-node out_dir) follows
        rank 0 instead of restarting the world from scratch.  An out_dir written before the
        tag existed (aggregate on disk, no tag) resumes from rank 0's sidecar
        ``completed_rounds``, with a warning.  A client's own ``clientN_model.pth`` is never the
        resume point of a collective run: after a crash inside a round it holds that round's
        LOCAL model (fed/runner.py run_round saves it before FedAvg).  Single-process runs with
        no sidecar keep the reference behaviour of loading it (client1.py:375-377: re-running
        the script is the next round)."""
        cfg, log = self.cfg, self.log
        st = ck.load_fed_state(cfg.out_dir, self.client_id)
        start = 0
        if self.di.is_main or not self.di.distributed:
            start = ck.load_global_round(cfg.out_dir)
            legacy = int((st or {}).get("completed_rounds", 0))
            if start == 0 and os.path.exists(ck.global_ckpt_path(cfg.out_dir)):
                if legacy > 0:
                    log.info(f"[WARN] {ck.global_ckpt_path(cfg.out_dir)} has no round tag (written by an older "
                             f"version): resuming from the client sidecar's {legacy} completed round(s)")
                    start = legacy
                else:
                    log.info(f"[WARN] {ck.global_ckpt_path(cfg.out_dir)} has no round tag and no sidecar "
                             f"records a completed round: starting from round 1")
        if self.di.distributed:
            start = int(comm.broadcast_float(float(start), src=0))
        if start > 0:
            path = ck.global_ckpt_path(cfg.out_dir)
            if self.di.is_main or not self.di.distributed:
                ck.load_model(self.model, path)
            broadcast_model(self.model, comm=self.comm)
            self.start_round = start
            self.history = [h for h in (st or {}).get("history", []) if int(h.get("round", 0)) <= start]
            done = int((st or {}).get("completed_rounds", 0))
            if done != start:
                log.info(f"client sidecar says {done} completed round(s); the aggregate says {start}")
            log.info(f"loading pre-trained model from {path} (aggregate of round {start})")
        elif st is None and not self.di.distributed:
            path = ck.client_ckpt_path(cfg.out_dir, self.client_id)
            if ck.load_model(self.model, path):
                log.info(f"loading pre-trained model from {path}")

    # ------------------------------------------------------------------ one round
    def run_round(self, r: int) -> Dict:
        cfg, log, model = self.cfg, self.log, self.model
        log.phase(f"Starting round {r + 1}/{cfg.rounds}")
        opt = ArenaAdam(model, lr=cfg.lr, betas=cfg.betas, eps=cfg.eps, weight_decay=cfg.weight_decay,
                        decoupled=cfg.decoupled_weight_decay)
        opt.reset_state()  # a fresh Adam every round (client1.py:380), "has state" row flags included
        opt_path = os.path.join(cfg.out_dir, f"client{self.client_id}_optim.pth")
        if cfg.save_optimizer and r == self.start_round:
            ck.load_optimizer(opt, opt_path)
        teacher_test = None
        if self.teacher is not None and r == self.start_round:
            # Local teacher fine-tune (BERT-base, same kernels), then distil into the student.
            log.info("training BERT-base teacher")
            t_opt = ArenaAdam(self.teacher, lr=cfg.lr)
            with self.timer("teacher"):
                train_model(self.teacher, self.train_loader, None, t_opt, int(cfg.extra.get("teacher_epochs", cfg.epochs)),
                            log=log, use_graph=cfg.use_graph and (self.teacher_sync is None or cfg.dp_graph
                                                                  or self.teacher_sync.capturable),
                            grad_sync=self.teacher_sync)
            with self.timer("eval"):
                teacher_test = _metrics_record(evaluate_model(self.teacher, self.test_loader, log=log,
                                                              name="Teacher test"))
            self.teacher.eval()
        with self.timer("train"):
            use_graph = cfg.use_graph and (self.grad_sync is None or cfg.dp_graph or self.grad_sync.capturable)
            tr = train_model(model, self.train_loader, None, opt, cfg.epochs, log=log, use_graph=use_graph,
                             teacher=self.teacher, kd_temperature=cfg.kd_temperature, kd_alpha=cfg.kd_alpha,
                             grad_sync=self.grad_sync)
        log.info("evaluating local model on validation set...")
        with self.timer("eval"):
            val_local = evaluate_model(model, self.val_loader, log=log, name="Validation")
            log.info("evaluating local model on test set...")
            local = evaluate_model(model, self.test_loader, log=log, name="Test")
        sfx = "" if r == 0 else f"_round{r + 1}"
        if self.writer:
            save_metrics(local, os.path.join(cfg.out_dir, f"client{self.client_id}_local_metrics{sfx}.csv"), log)
            if cfg.save_checkpoints:
                ck.save_model(model, ck.client_ckpt_path(cfg.out_dir, self.client_id))
            if cfg.save_optimizer:
                ck.save_optimizer(opt, opt_path)

        # ---- FedAvg (replaces send_model -> server aggregate -> receive_aggregated_model)
        part = faults.participants(r, self.num_clients, cfg.participation, cfg.base_seed)
        contributes = self.idx in part and not faults.dropped(cfg, self.idx, r)
        weight = float(len(self.data.train)) if cfg.weighted_fedavg else 1.0
        weight /= self.topo.gpus_per_client  # k identical replicas per client share its weight
        faults.maybe_kill(self.idx, r, cfg.out_dir, self.topo.dp_rank, phase="fedavg")
        if self.health is not None:
            try:  # every client alive and here, or fail fast naming the dead rank
                self.health.barrier(f"fedavg/{r}")
            except health.PeerFailure as e:
                log.info(f"[ERROR] {e}; aborting round {r + 1} (restart resumes from the last completed round)")
                raise
        with self.timer("fedavg"):
            t0 = time.perf_counter()
            if cfg.transport == "tcp":
                # one upload per client (its replica 0, as the reference's one process per
                # client); the other replicas take the aggregate from it
                total_w = self._tcp_exchange(contributes) if self.topo.dp_rank == 0 else 0.0
                if self.topo.dp:
                    total_w = self._dp_share_model(total_w)
            else:
                total_w = fedavg_(model, weight=weight, participate=contributes, comm=self.comm)
            if model.device.type == "cuda":
                torch.cuda.synchronize()
            t_fed = time.perf_counter() - t0
        log.info(f"updated with aggregated model (participated={contributes}, total weight={total_w:g}, "
                 f"{t_fed * 1e3:.2f} ms)")
        if self.di.is_main and cfg.save_checkpoints:
            ck.save_global(model, cfg.out_dir, r + 1)  # weights, then the round tag (_resume)
        faults.maybe_kill(self.idx, r, cfg.out_dir, self.topo.dp_rank, phase="post_fedavg")
        log.info("evaluating aggregated model on validation set...")
        with self.timer("eval"):
            val_agg = evaluate_model(model, self.val_loader, log=log, name="Validation")
            log.info("evaluating aggregated model on test set...")
            agg = evaluate_model(model, self.test_loader, log=log, name="Test")
        if self.writer:
            save_metrics(agg, os.path.join(cfg.out_dir, f"client{self.client_id}_aggregated_metrics{sfx}.csv"), log)
        if cfg.plots and self.writer:
            with self.timer("plot"):
                from ..utils.plots import plot_evaluation, reference_dpi
                dpi = cfg.plot_dpi if cfg.plot_dpi > 0 else reference_dpi(self.client_id)
                plot_evaluation(local, agg, os.path.join(cfg.out_dir, f"client{self.client_id}_plots"),
                                f"Client {self.client_id}", dpi=dpi, log=log)
        if self.writer and cfg.save_checkpoints:
            ck.save_model(model, ck.client_ckpt_path(cfg.out_dir, self.client_id))
        rec = {"round": r + 1, "train": tr, "fedavg_ms": t_fed * 1e3, "participated": contributes,
               "local_val": _metrics_record(val_local), "local_test": _metrics_record(local),
               "aggregated_val": _metrics_record(val_agg), "aggregated_test": _metrics_record(agg)}
        if teacher_test is not None:
            rec["teacher_test"] = teacher_test
        self.history.append(rec)
        if self.writer:
            ck.save_fed_state(cfg.out_dir, self.client_id, {"completed_rounds": r + 1, "history": self.history})
        return rec

    def _tcp_exchange(self, contributes: bool) -> float:
        """Reference protocol: upload to the FedAvg server, download the mean (client1.py:391-395)."""
        from ..parallel import transport as tp
        cfg, log = self.cfg, self.log
        if contributes:
            ok = tp.send_model(self.model.state_dict(), cfg.server_host, cfg.port_receive, cfg.gzip_level,
                               cfg.timeout_s, log)
            if not ok:
                log.info("skipping aggregated model evaluation due to send failure")
                return 0.0
        agg = tp.receive_aggregated_model(cfg.server_host, cfg.port_send, timeout=cfg.timeout_s, log=log)
        if agg is None:
            log.info("skipping aggregated model evaluation due to connection failure")
            return 0.0
        self.model.load_state_dict(agg)
        return float(self.num_clients)

    def _dp_share_model(self, total_w: float) -> float:
        """Replica 0 of this client -> the client's other replicas: weights + FedAvg weight."""
        import torch.distributed as dist
        A = self.model.arena
        src = self.topo.client_ranks(self.topo.client_idx)[0]
        dist.broadcast(A.master, src=src, group=self.topo.dp_group)
        t = torch.tensor([total_w], dtype=torch.float64, device=A.device)
        dist.broadcast(t, src=src, group=self.topo.dp_group)
        if hasattr(self.model, "sync_shadow"):
            self.model.sync_shadow(force=True)
        return float(t.item())

    # ------------------------------------------------------------------ all rounds
    def run(self) -> Dict:
        self.setup()
        try:
            for r in range(self.start_round, self.cfg.rounds):
                self.run_round(r)
            report = self.report()
        finally:
            health.stop()
        self.log.phase("Client shutdown")
        return report

    def report(self) -> Dict:
        """Cross-client summary on rank 0 (gathered with an all-gather of small vectors)."""
        last = self.history[-1] if self.history else None
        vec = [0.0] * 8
        if last:
            a, l_ = last["aggregated_test"], last["local_test"]
            vec = [a["accuracy"], a["f1"], a["precision"], a["recall"], l_["accuracy"], l_["f1"],
                   last["train"]["batches_per_sec"], last["fedavg_ms"]]
        allv = comm.all_gather_floats(vec)[::self.topo.gpus_per_client]  # replica 0 of each client
        rep = {"clients": [{"client": i + 1, "aggregated_test_accuracy": v[0], "aggregated_test_f1": v[1],
                            "aggregated_test_precision": v[2], "aggregated_test_recall": v[3],
                            "local_test_accuracy": v[4], "local_test_f1": v[5], "train_batches_per_sec": v[6],
                            "fedavg_ms": v[7]} for i, v in enumerate(allv)],
               "rounds": self.cfg.rounds, "world_size": self.di.world_size,
               "gpus_per_client": self.topo.gpus_per_client, "phases_s": self.timer.summary()}
        if self.di.is_main:
            path = os.path.join(self.cfg.out_dir, "federated_report.json")
            with open(path, "w") as f:
                json.dump(rep, f, indent=1)
            self.log.info(f"federated report written to {path}")
        return rep


@torch.no_grad()
def _average_masters(model, states: List[torch.Tensor]) -> None:
    """``fedavg_``'s arithmetic in one process: the SUM of the clients' fp32 masters (what the
    all-reduce computes; for two clients a + b is exact in any order), then the fused 1/N scale +
    bf16 shadow refresh (``scale_cast``) on GPU."""
    A = model.arena
    A.master.copy_(states[0])
    for s in states[1:]:
        A.master.add_(s)
    if A.master.is_cuda:
        from ..ops import kernels as K
        K.scale_cast(A.master, A.shadow, 1.0 / len(states))
        model.mark_shadow_synced()
    else:
        A.master.mul_(1.0 / len(states))
        model.sync_shadow(force=True)


def warm_start(client: "FederatedClient", epochs: int = 1, rows: int = 225_745, seed: int = 1,
               profile: str = "default", fraction: float = 0.1) -> Dict:
    """A shared "pretrained" starting point for every client (the reference fine-tunes a PRETRAINED
    DistilBERT, client1.py:56, so its clients start near one point; no weights can be downloaded
    here): ``client.model`` is trained ``epochs`` epochs on a public synthetic sample -- a separate
    file (generator seed ``seed``, profile ``profile``) that no client samples from -- with a fresh
    Adam.  The model's dropout counters are then reset, so the federated clients start exactly as
    they would from a loaded checkpoint.  Returns the training record and the public test metrics."""
    cfg, model = client.cfg, client.model
    frame = generate_cicids2017(rows, seed=seed, profile=profile)
    data = build_client_data(frame, 0, fraction, cfg.base_seed + 1000, cfg.max_len, client.tokenizer)
    dev = model.device
    loader = DeviceLoader(data.train, cfg.batch_size, shuffle=True, device=dev, seed=cfg.base_seed + 1000)
    opt = ArenaAdam(model, lr=cfg.lr, betas=cfg.betas, eps=cfg.eps, weight_decay=cfg.weight_decay,
                    decoupled=cfg.decoupled_weight_decay)
    opt.reset_state()
    tr = train_model(model, loader, None, opt, epochs, log=client.log, use_graph=cfg.use_graph)
    test = _metrics_record(evaluate_model(model, DeviceLoader(data.test, cfg.eval_batch_size, device=dev),
                                          name="Public warm-start test"))
    opt.reset_state()  # (also clears the "has Adam state" word-row flags)
    with torch.no_grad():
        model.rng.zero_()
    model.torch_counter = 0
    return {"train": tr, "public_test": test, "rows": rows, "seed": seed, "profile": profile,
            "train_rows": len(data.train)}


def _pooled(recs, key: str):
    return [[sum(r[key]["confusion_matrix"][i][j] for r in recs if len(r[key]["confusion_matrix"]) == 2)
             for j in range(2)] for i in range(2)]


def run_virtual_clients(client: "FederatedClient", n_clients: int = 2, rounds: int = 1,
                        progress=None) -> Dict:
    """``rounds`` FedAvg rounds of ``n_clients`` federated clients on THIS process's device, the
    clients trained one after another (a 1-GPU job: ``bench.py`` quality half with
    ``--virtual-clients N --rounds R``, ``cli launch --virtual-clients``).

    Reference protocol (client1.py / client2.py + server.py:67-79): client k samples its own 10 %
    of the file with seed 42 + k (client1.py:89, client2.py:84), every client starts from the same
    weights (round 1: the model's broadcast init; round r > 1: round r-1's aggregate --
    the reference's next round is a re-run of the scripts that loads the aggregate,
    client1.py:375-377), trains ``cfg.epochs`` local epochs with a FRESH Adam (client1.py:380
    re-creates it every run), is evaluated on its test split, the server averages the fp32 state
    dicts (unweighted mean; ``_average_masters`` = fedavg_'s sum + ``scale_cast``) and every client
    then evaluates the aggregate on its own test split (client1_aggregated_metrics.csv).

    Each virtual client keeps, across rounds, exactly the state a real client process keeps in
    ``FederatedClient.run`` (one process per client): its shuffling loader (the epoch permutations
    continue) and its dropout counters (``model.rng`` / ``torch_counter``), so for the same config
    the R-round virtual run equals the N-rank collective ``run_federated`` run bit for bit
    (tests/test_virtual_rounds.py, N = 2, R = 2 on gloo).

    Returns ``rounds`` (one record per round: per-client local / aggregated metrics, the pooled
    aggregated confusion, the FedAvg time) plus the LAST round's ``clients`` /
    ``aggregated_confusion`` / ``fedavg_ms`` at the top level (the 1-round API of earlier rounds).

    With a teacher (the distillation extension, BASELINE.json config 5) every virtual client does
    what ``run_round`` does for a real one: in its first round the shared BERT-base teacher init is
    fine-tuned on the client's own split (``teacher_epochs``) and kept for the later rounds (the
    teachers stay local, as in run_round), then the client's student is distilled from it; the
    students are averaged.  Each first-round record then also holds the client's ``teacher_test``."""
    cfg, model = client.cfg, client.model
    if client.di.distributed:
        raise RuntimeError("virtual clients run in a single-process job (world size 1)")
    teacher = client.teacher
    dev = model.device
    A = model.arena
    glob = A.master.detach().clone()  # what every client starts the round from
    t_init = teacher.arena.master.detach().clone() if teacher is not None else None
    say = progress or (lambda msg: None)
    # per-client state that survives the rounds (a real client's process keeps it)
    cs = []
    for v in range(n_clients):
        data = build_client_data(client.frame, v, cfg.data_fraction, cfg.base_seed, cfg.max_len, client.tokenizer,
                                 cfg.partition, n_clients)
        cs.append({"data": data,
                   "loader": DeviceLoader(data.train, cfg.batch_size, shuffle=True, device=dev,
                                          seed=cfg.client_seed(v)),
                   "test": DeviceLoader(data.test, cfg.eval_batch_size, device=dev),
                   "rng": model.rng.detach().clone(), "torch_counter": model.torch_counter, "teacher": None})
    hist = []
    for r in range(rounds):
        locals_, recs = [], []
        for v, c in enumerate(cs):
            data, loader, test = c["data"], c["loader"], c["test"]
            rec = {"client": v + 1, "round": r + 1, "train_rows": len(data.train), "test_rows": len(data.test)}
            t0 = time.perf_counter()
            if teacher is not None:
                if c["teacher"] is None:
                    with torch.no_grad():
                        teacher.arena.master.copy_(t_init)
                    teacher.sync_shadow(force=True)
                    t_opt = ArenaAdam(teacher, lr=cfg.lr)
                    t_opt.reset_state()
                    teacher.train()
                    rec["teacher_train"] = train_model(
                        teacher, loader, None, t_opt, int(cfg.extra.get("teacher_epochs", cfg.epochs)),
                        log=client.log, use_graph=cfg.use_graph)
                    rec["teacher_test"] = _metrics_record(evaluate_model(teacher, test,
                                                                         name=f"Client {v + 1} teacher test"))
                    c["teacher"] = teacher.arena.master.detach().clone()
                    del t_opt
                else:
                    with torch.no_grad():
                        teacher.arena.master.copy_(c["teacher"])
                    teacher.sync_shadow(force=True)
                teacher.eval()
            with torch.no_grad():
                A.master.copy_(glob)
                model.rng.copy_(c["rng"])
            model.torch_counter = c["torch_counter"]
            model.sync_shadow(force=True)
            opt = ArenaAdam(model, lr=cfg.lr, betas=cfg.betas, eps=cfg.eps, weight_decay=cfg.weight_decay,
                            decoupled=cfg.decoupled_weight_decay)
            opt.reset_state()  # (also clears the sparse word rows' "has Adam state" flags)
            tr = train_model(model, loader, None, opt, cfg.epochs, log=client.log, use_graph=cfg.use_graph,
                             teacher=teacher, kd_temperature=cfg.kd_temperature, kd_alpha=cfg.kd_alpha)
            with torch.no_grad():
                c["rng"].copy_(model.rng)
            c["torch_counter"] = model.torch_counter
            local = _metrics_record(evaluate_model(model, test, name=f"Client {v + 1} local test"))
            locals_.append(A.master.detach().clone())
            rec.update({"train": tr, "train_wall_s": time.perf_counter() - t0, "local_test": local})
            recs.append(rec)
            del opt
            say(f"round {r + 1}/{rounds} client {v + 1}/{n_clients}: local acc {local['accuracy']:.3f} % "
                f"f1 {local['f1']:.5f} ({tr['steps']} steps, {time.perf_counter() - t0:.1f} s)")
        t0 = time.perf_counter()
        _average_masters(model, locals_)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        fed_ms = 1e3 * (time.perf_counter() - t0)
        agg = A.master.detach()
        for rec, c, loc in zip(recs, cs, locals_):
            rec["aggregated_test"] = _metrics_record(evaluate_model(model, c["test"], name=f"Client {rec['client']} "
                                                                                           "aggregated test"))
            rec["rel_l2_local_to_aggregate"] = float((loc - agg).norm() / loc.norm().clamp_min(1e-30))
        glob = agg.clone()
        del locals_
        pooled = _pooled(recs, "aggregated_test")
        hist.append({"round": r + 1, "clients": recs, "fedavg_ms": fed_ms, "aggregated_confusion": pooled,
                     "local_confusion": _pooled(recs, "local_test")})
        (tn, fp), (fn, tp) = pooled
        say(f"round {r + 1}/{rounds} aggregate: pooled acc {100.0 * (tp + tn) / max(tp + tn + fp + fn, 1):.3f} %")
    last = hist[-1]
    return {"clients": last["clients"], "fedavg_ms": last["fedavg_ms"],
            "aggregated_confusion": last["aggregated_confusion"], "rounds": hist}


def run_federated(cfg: FedConfig, frame=None, model_config: Optional[DistilBertConfig] = None) -> Dict:
    client = FederatedClient(cfg, frame, model_config)
    try:
        return client.run()
    finally:
        client.log.close()
