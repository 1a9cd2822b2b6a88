"""Checkpoints with the reference's file names and key layout + a round sidecar.

Reference: each client ``torch.save(model.state_dict(), 'clientN_model.pth')``
after local training (client1.py:388) and after loading the aggregate (:403);
on start it loads that file if present (:375-377) -> re-running = next round.
The server writes the averaged dict to ``ddos_distilbert_model.pth`` (server.py:77).

Added here: ``fed_state.json`` (completed round index, config digest, metrics
history) so ``--resume`` continues at the right round, and an optional
optimizer sidecar.  Loading always uses ``weights_only=True``.
"""
from __future__ import annotations

import json
import os
import tempfile
from typing import Dict, Optional

import torch


def client_ckpt_path(out_dir: str, client_id: int) -> str:
    return os.path.join(out_dir, f"client{client_id}_model.pth")


def global_ckpt_path(out_dir: str) -> str:
    return os.path.join(out_dir, "ddos_distilbert_model.pth")


def state_path(out_dir: str, client_id: int) -> str:
    return os.path.join(out_dir, f"client{client_id}_fed_state.json")


def _atomic_save(obj, path: str):
    d = os.path.dirname(path) or "."
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(dir=d, suffix=".tmp")
    os.close(fd)
    torch.save(obj, tmp)
    os.replace(tmp, path)


def save_model(model, path: str):
    """fp32 state_dict with the reference's 102 keys, CPU tensors (portable)."""
    sd = {k: v.detach().to("cpu", torch.float32).clone() for k, v in model.state_dict().items()}
    _atomic_save(sd, path)
    return path


def load_model(model, path: str, strict: bool = True) -> bool:
    if not os.path.exists(path):
        return False
    sd = torch.load(path, map_location="cpu", weights_only=True)
    model.load_state_dict(sd, strict=strict)
    return True


def global_tag_path(out_dir: str) -> str:
    return os.path.join(out_dir, "ddos_distilbert_model.json")


def save_global(model, out_dir: str, round_done: int) -> str:
    """Rank 0: the round-``round_done`` aggregate, then its round tag (written after the
    weights, so a tag never names a checkpoint that is not on disk yet)."""
    path = save_model(model, global_ckpt_path(out_dir))
    tag = global_tag_path(out_dir)
    with open(tag + ".tmp", "w") as f:
        json.dump({"round": int(round_done)}, f)
    os.replace(tag + ".tmp", tag)
    return path


def load_global_round(out_dir: str) -> int:
    """Round whose aggregate ``ddos_distilbert_model.pth`` holds (0: none / untagged)."""
    tag = global_tag_path(out_dir)
    if not (os.path.exists(tag) and os.path.exists(global_ckpt_path(out_dir))):
        return 0
    try:
        with open(tag) as f:
            return int(json.load(f).get("round", 0))
    except (OSError, ValueError):
        return 0


def save_optimizer(opt, path: str):
    _atomic_save(opt.state_dict(), path)


def load_optimizer(opt, path: str) -> bool:
    if not os.path.exists(path):
        return False
    opt.load_state_dict(torch.load(path, map_location="cpu", weights_only=True))
    return True


def save_fed_state(out_dir: str, client_id: int, state: Dict):
    path = state_path(out_dir, client_id)
    os.makedirs(out_dir, exist_ok=True)
    with open(path + ".tmp", "w") as f:
        json.dump(state, f, indent=1, default=float)
    os.replace(path + ".tmp", path)


def load_fed_state(out_dir: str, client_id: int) -> Optional[Dict]:
    path = state_path(out_dir, client_id)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)
