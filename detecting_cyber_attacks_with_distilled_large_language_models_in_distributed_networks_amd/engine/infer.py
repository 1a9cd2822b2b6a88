"""Inference / serving path: classify flow records with a trained DDoSClassifier.

The reference only evaluates inside the training script (client1.py:118-150,
8.9-14 batches/s at bs16 in eager fp32).  For deployment the forward is the
same fused HIP path as training -- unpadded blocks, varlen attention -- and is
replayed as a HIP graph, one per (batch shape, packed-row bucket): a batch is
a handful of host copies plus one graph launch, with no host sync until the
caller reads the results.
"""
from __future__ import annotations

import time
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from ..data.dataset import short_batch
from .graph import contiguous_block, key_tokens, no_gc, static_block


class GraphedForward:
    """No-grad logits of ``model`` replayed from HIP graphs (eager on CPU / torch impl)."""

    def __init__(self, model, enabled: bool = True, max_graphs: int = 16):
        self.model = model
        self.enabled = enabled and model.device.type == "cuda" and getattr(model, "impl", "") == "hip"
        self.max_graphs = max_graphs
        self.graphs: Dict[tuple, tuple] = {}
        self.failed: Optional[str] = None

    def _key(self, ids, tokens):
        if tokens is None or not hasattr(self.model, "packed_rows"):
            return tuple(ids.shape), None, False
        return (tuple(ids.shape), int(self.model.packed_rows(tokens, ids.shape[0], ids.shape[1])),
                short_batch(tokens, ids.shape[1]))

    @torch.no_grad()
    def __call__(self, ids: torch.Tensor, mask: torch.Tensor, tokens: Optional[int] = None) -> torch.Tensor:
        m = self.model
        if m.training:
            m.eval()
        if not self.enabled or self.failed:
            return m(ids, mask, tokens=tokens)
        key = self._key(ids, tokens)
        hit = self.graphs.get(key)
        if hit is not None:
            # weights changed outside the optimizer (load_state_dict, FedAvg) -> refresh the
            # bf16 shadow the graph reads (host-side version check, a launch only when stale)
            if hasattr(m, "sync_shadow"):
                m.sync_shadow()
            g, static, out = hit
            blk = contiguous_block(ids, mask) if static["flat"] is not None else None
            if blk is not None:
                static["flat"].copy_(blk)
            else:
                static["ids"].copy_(ids)
                static["mask"].copy_(mask)
            g.replay()
            return out
        if len(self.graphs) >= self.max_graphs:
            return m(ids, mask, tokens=tokens)
        (s_ids, s_mask), flat = static_block(ids, mask)
        static = {"ids": s_ids, "mask": s_mask, "flat": flat}
        # one eager pass on a side stream warms the allocator / workspaces before capture
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m(static["ids"], static["mask"], tokens=key_tokens(key))
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        try:
            torch.cuda.synchronize()
            with no_gc(), torch.cuda.graph(g):
                out = m(static["ids"], static["mask"], tokens=key_tokens(key))
        except Exception as e:  # pragma: no cover - capture support varies by op
            self.failed = f"{type(e).__name__}: {e}"
            torch.cuda.synchronize()
            return m(ids, mask, tokens=tokens)
        self.graphs[key] = (g, static, out)
        g.replay()
        return out


@torch.no_grad()
def predict(model, loader, graphed: bool = True) -> Tuple[np.ndarray, np.ndarray, Dict]:
    """(P(DDoS) per row, predicted label per row, timing) over a DeviceLoader (no shuffle)."""
    fwd = GraphedForward(model, enabled=graphed)
    dev = model.device
    n = loader.n
    probs = torch.empty(n, dtype=torch.float32, device=dev)
    preds = torch.empty(n, dtype=torch.int64, device=dev)
    off = nb = 0
    t0 = time.perf_counter()
    for batch in loader:
        logits = fwd(batch["input_ids"], batch["attention_mask"], batch.get("n_tokens")).float()
        b = logits.shape[0]
        probs[off:off + b] = torch.softmax(logits, dim=1)[:, 1]
        preds[off:off + b] = (logits[:, 1] > logits[:, 0]).long()  # ties -> 0, as torch.max picks the first
        off += b
        nb += 1
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    timing = {"rows": off, "batches": nb, "seconds": dt, "rows_per_sec": off / dt if dt > 0 else 0.0,
              "batches_per_sec": nb / dt if dt > 0 else 0.0, "graphs": len(fwd.graphs), "graph_error": fwd.failed}
    return probs[:off].cpu().numpy(), preds[:off].cpu().numpy(), timing
