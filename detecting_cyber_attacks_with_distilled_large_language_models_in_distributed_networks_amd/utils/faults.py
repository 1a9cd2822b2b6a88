"""Fault injection for the federated round loop (the reference has none).

Knobs (config fields or env):
  drop_client / drop_round   drop client k's update at round r (it still receives the aggregate)
  FEDDDOS_KILL_CLIENT=k, FEDDDOS_KILL_ROUND=r
                              hard-exit client k at the start of round r's FedAvg
                              (surviving ranks then hit the collective timeout)
  participation < 1.0         seeded partial participation: each round a subset of
                              clients of size max(1, round(p*N)) contributes
"""
from __future__ import annotations

import os
import random
from typing import List


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


def maybe_kill(client_idx: int, round_idx: int):
    k = os.environ.get("FEDDDOS_KILL_CLIENT")
    r = os.environ.get("FEDDDOS_KILL_ROUND")
    if k is not None and int(k) == client_idx and (r is None or int(r) == round_idx):
        os._exit(17)
