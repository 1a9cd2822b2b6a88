"""Fault injection for the federated round loop (the reference has none).

Knobs (config fields or env):
  drop_client / drop_round   drop client k's update at round r (it still receives the aggregate)
  FEDDDOS_KILL_CLIENT=k, FEDDDOS_KILL_ROUND=r, FEDDDOS_KILL_AT=fedavg|post_fedavg
                              hard-exit client k at the start of round r's FedAvg (default),
                              or after it (aggregate written by rank 0, before the client
                              records the round in its fed_state sidecar); the
                              survivors' health-checked barrier (parallel/health.py) names
                              the dead rank within seconds.  One-shot per (k, r) when a
                              marker directory is given, so an elastic restart
                              (torchrun --max-restarts) of the same round succeeds.
  participation < 1.0         seeded partial participation: each round a subset of
                              clients of size max(1, round(p*N)) contributes
"""
from __future__ import annotations

import os
import random
from typing import List, Optional


def participants(round_idx: int, num_clients: int, fraction: float, seed: int = 0) -> List[int]:
    """0-based client indices that contribute to ``round_idx`` (same on every rank)."""
    if fraction >= 1.0:
        return list(range(num_clients))
    k = max(1, int(round(fraction * num_clients)))
    rng = random.Random(seed * 1_000_003 + round_idx)
    return sorted(rng.sample(range(num_clients), k))


def dropped(cfg, client_idx: int, round_idx: int) -> bool:
    return cfg.drop_client is not None and cfg.drop_client == client_idx and \
        (cfg.drop_round is None or cfg.drop_round == round_idx)


def maybe_kill(client_idx: int, round_idx: int, marker_dir: Optional[str] = None, replica: int = 0,
               phase: str = "fedavg"):
    k = os.environ.get("FEDDDOS_KILL_CLIENT")
    r = os.environ.get("FEDDDOS_KILL_ROUND")
    if os.environ.get("FEDDDOS_KILL_AT", "fedavg") != phase:
        return
    if k is not None and int(k) == client_idx and (r is None or int(r) == round_idx):
        if marker_dir is not None:
            marker = os.path.join(marker_dir, f".killed_client{client_idx}_round{round_idx}_r{replica}")
            if os.path.exists(marker):
                return
            open(marker, "w").close()
        os._exit(17)
