"""Typed run configuration: one dataclass + CLI flags + env overrides.

The reference has no config system; its literals live in module constants and
inside ``main`` (client1.py:22-23, :356-358, :370-372, :380; server.py:10-13).
Every such literal becomes a field here whose default is the reference value,
so "parity mode" needs no flags.  Per-client variation (client2.py is a copy of
client1.py with seed 43) is derived from the rank: ``seed = base_seed + client_id``.

Env overrides: any field can be set with ``FEDDDOS_<FIELD>`` (upper case).
"""
from __future__ import annotations

import argparse
import dataclasses
import os
from dataclasses import dataclass, field
from typing import Optional


@dataclass
class FedConfig:
    # --- data (client1.py:23, :84-93, :356) -------------------------------------------
    csv_path: Optional[str] = None          # None -> synthetic CICIDS2017-shaped data
    synthetic_rows: int = 225_745           # full Friday-DDoS file size
    # synthetic generator setting (data/synthetic.py PROFILES): "default" (saturates near 99.95 %),
    # "calibrated" (local models near the reference's 99.05 %), "hard" (numerics tests, ~95 %)
    data_profile: str = "default"
    data_fraction: float = 0.1              # client1.py:23
    base_seed: int = 42                     # client1.py:89 (client2.py:84 uses 43)
    partition: str = "iid_overlap"          # "iid_overlap" (reference) | "disjoint"
    max_len: int = 128                      # client1.py:27
    # --- model (client1.py:53-65) ---------------------------------------------------
    model_path: Optional[str] = None        # optional HF distilbert dir; None -> random init
    head_dropout: float = 0.3               # client1.py:57
    hidden_dropout: float = 0.1
    attention_dropout: float = 0.1
    # --- training (client1.py:370-380) ------------------------------------------------
    batch_size: int = 16                    # client1.py:370 (bench uses 32, BASELINE.json)
    eval_batch_size: int = 16
    epochs: int = 3                         # client1.py:380
    lr: float = 2e-5                        # client1.py:380
    betas: tuple = (0.9, 0.999)
    eps: float = 1e-8
    weight_decay: float = 0.0
    decoupled_weight_decay: bool = False    # AdamW when True
    impl: str = "auto"                      # "hip" | "torch" | "auto" (hip on GPU)
    use_graph: bool = True                  # capture the train step in a HIP graph
    # --- federation (server.py:10-13) -------------------------------------------------
    rounds: int = 1
    num_clients: Optional[int] = None       # None -> world size / gpus_per_client
    gpus_per_client: int = 1                # >1: each client is k data-parallel GPUs (parallel/dp.py)
    dp_graph: bool = False                  # capture data-parallel steps (collectives) in the HIP graph
    weighted_fedavg: bool = False           # reference is unweighted (server.py:73-76)
    participation: float = 1.0              # fraction of clients aggregated per round
    timeout_s: float = 300.0                # server.py:10 / client1.py:22
    heartbeat_s: float = 1.0                # failure detection (parallel/health.py); 0 disables
    heartbeat_stale_s: float = 10.0         # a peer silent this long is declared dead
    transport: str = "collective"           # "collective" (RCCL/gloo all-reduce) | "tcp" (reference framing; weights-only payload)
    comm: str = "torch"                     # collective backend: "torch" (torch.distributed) | "rccl" (NativeComm)
    server_host: str = "localhost"          # client1.py:276,314
    port_receive: int = 12345               # server.py:11
    port_send: int = 12346                  # server.py:12
    gzip_level: int = 1                     # tcp payload compression (reference: 9)
    # --- outputs ------------------------------------------------------------------------
    out_dir: str = "."
    plots: bool = True
    plot_dpi: int = 0                       # 0: reference per-client DPI (client 1 default, client 2: 300)
    resume: bool = True                     # client1.py:375-377 loads clientN_model.pth
    save_optimizer: bool = False
    save_checkpoints: bool = True           # clientN_model.pth / ddos_distilbert_model.pth (bench: off)
    # --- fault injection -------------------------------------------------
    drop_client: Optional[int] = None       # client whose update is dropped ...
    drop_round: Optional[int] = None        # ... at this round
    # --- distillation extension (BASELINE.json config 5) ------------------------------
    teacher: Optional[str] = None           # "bert-base" -> KD from a 12-layer teacher
    kd_temperature: float = 2.0
    # loss = alpha CE + (1 - alpha) T^2 KL(teacher || student).  Measured on the config-5 protocol
    # (seq256 bs64, 3 teacher + 3 student epochs, 4,515 test rows; profiles/r3_kd_sweep.txt):
    # alpha 0.5 -> student F1 0.9888, 0.9 -> 0.9988 (teacher 0.9990)
    kd_alpha: float = 0.9
    verbose: bool = True
    extra: dict = field(default_factory=dict)

    def client_seed(self, client_id: int) -> int:
        return self.base_seed + client_id

    @classmethod
    def from_env(cls, base: Optional["FedConfig"] = None) -> "FedConfig":
        cfg = base or cls()
        for f in dataclasses.fields(cls):
            key = "FEDDDOS_" + f.name.upper()
            if key in os.environ:
                setattr(cfg, f.name, _coerce(f, os.environ[key], getattr(cfg, f.name)))
        return cfg

    @classmethod
    def add_cli(cls, parser: argparse.ArgumentParser) -> argparse.ArgumentParser:
        for f in dataclasses.fields(cls):
            if f.name == "extra":
                continue
            name = "--" + f.name.replace("_", "-")
            default = f.default if f.default is not dataclasses.MISSING else None
            if isinstance(default, bool):
                parser.add_argument(name, dest=f.name, default=None,
                                    type=lambda s: s.lower() in ("1", "true", "yes", "on"),
                                    metavar="BOOL")
            elif isinstance(default, tuple):
                parser.add_argument(name, dest=f.name, default=None, type=float, nargs=len(default))
            else:
                typ = type(default) if default is not None else str
                if f.name in ("drop_client", "drop_round", "num_clients"):
                    typ = int
                parser.add_argument(name, dest=f.name, default=None, type=typ)
        return parser

    @classmethod
    def from_args(cls, ns: argparse.Namespace) -> "FedConfig":
        cfg = cls.from_env()
        for f in dataclasses.fields(cls):
            v = getattr(ns, f.name, None)
            if v is not None:
                setattr(cfg, f.name, tuple(v) if isinstance(f.default, tuple) else v)
        return cfg


def _coerce(f, raw: str, current):
    if isinstance(current, bool):
        return raw.lower() in ("1", "true", "yes", "on")
    if isinstance(current, int):
        return int(raw)
    if isinstance(current, float):
        return float(raw)
    if isinstance(current, tuple):
        return tuple(float(x) for x in raw.split(","))
    if current is None and f.name in ("drop_client", "drop_round", "num_clients"):
        return int(raw)
    return raw
