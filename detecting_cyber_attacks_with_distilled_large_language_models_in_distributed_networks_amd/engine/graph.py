"""HIP-graph capture of the whole training step (forward + backward + Adam).

At B32/S128 one step is ~150 kernel launches; replaying them as one hipGraph
removes the per-launch host cost and all Python/autograd overhead from the
steady state (the MI355X replacement for a tracing compiler).  The dropout
seed counter and the Adam step count live on the device and are advanced by
kernels inside the graph, so every replay is a fresh, correct step.

Protocol: the first ``warmup`` calls run eagerly (they are real training steps
on the real batches, and they populate allocator pools / workspaces); the next
call captures, then replays the capture for its own batch.  Batches whose shape
differs from the captured one (the last partial batch, drop_last=False) run
eagerly.

``step_fn.prepare`` (optional): called eagerly before every replay and before the capture, for
state a replay does not refresh by itself -- the model's bf16 weight shadow after an out-of-band
write of its fp32 masters (a checkpoint load): the captured forward holds no shadow sync of its
own (models/distilbert.py prepare_replay).

Unpadded model path: a batch also carries its real-token count; ``bucket(tokens,
B, S)`` (the model's ``packed_rows``) maps it to the packed row count the step
is shaped by, and one graph is captured per (batch shape, bucket) -- a handful
for CICIDS2017 text (76-86 real tokens of 128).  Inside a graph everything that
depends on the actual batch (row maps, sequence starts) is computed on device
from the mask, so any batch of the same bucket replays it.
"""
from __future__ import annotations

import gc
from typing import Callable, Dict, Optional

import torch

from ..data.dataset import PackedTokens, short_batch
from ..ops.graph_split import GRAPH_SPLIT, _Capture, split_point  # noqa: F401


class no_gc:
    """Python's cyclic GC paused over a graph capture: a collection that runs mid-capture can free
    an unreachable model's HIP graphs / tensors (a model and its cached eval GraphedForward
    reference each other), and the resulting hipGraphExecDestroy / hipFree is not permitted while
    the stream captures (measured: scripts/curve_bisect.py's 8th model, round 4)."""

    def __enter__(self):
        self.was = gc.isenabled()
        gc.collect()
        gc.disable()
        return self

    def __exit__(self, *exc):
        if self.was:
            gc.enable()
        return False


def contiguous_block(*ts: torch.Tensor) -> Optional[torch.Tensor]:
    """A flat view over ``ts`` if they lie back to back in one storage with one dtype
    (DeviceLoader's batch layout: ids | mask | labels), else None -- lets a graph replay
    refresh its static inputs with ONE copy instead of one per tensor."""
    t0 = ts[0]
    es = t0.element_size()
    ptr = t0.data_ptr()
    for t in ts:
        if not t.is_contiguous() or t.dtype != t0.dtype or t.device != t0.device or t.data_ptr() != ptr:
            return None
        if t.untyped_storage().data_ptr() != t0.untyped_storage().data_ptr():
            return None
        ptr += t.numel() * es
    n = sum(t.numel() for t in ts)
    return torch.as_strided(t0, (n,), (1,))


def static_block(*ts: torch.Tensor):
    """Clones of ``ts`` laid out back to back in one buffer (+ that buffer), or plain clones
    (+ None) when the dtypes differ."""
    if any(t.dtype != ts[0].dtype for t in ts):
        return [t.clone() for t in ts], None
    flat = torch.empty(sum(t.numel() for t in ts), dtype=ts[0].dtype, device=ts[0].device)
    out, off = [], 0
    for t in ts:
        v = flat[off:off + t.numel()].view(t.shape)
        v.copy_(t)
        out.append(v)
        off += t.numel()
    return out, flat


def key_tokens(key):
    """The ``tokens`` a graph of this key is captured with: the bucket's packed-row count (the
    rows the replays run on), carrying max_len <= 128 when the key is a short batch's."""
    if key[1] is None:
        return None
    return PackedTokens(key[1], 128) if key[2] else int(key[1])


class GraphedTrainStep:
    def __init__(self, step_fn: Callable[..., torch.Tensor], warmup: int = 2, enabled: bool = True,
                 bucket: Optional[Callable[[int, int, int], int]] = None, max_graphs: int = 16):
        self.step_fn = step_fn
        self.warmup = warmup
        self.enabled = enabled and torch.cuda.is_available()
        self.bucket = bucket
        self.max_graphs = max_graphs
        self.calls = 0
        self.graphs: Dict[tuple, tuple] = {}  # key -> (graph chain, static inputs, static loss)
        self.failed: Optional[str] = None
        self.split = GRAPH_SPLIT
        self._stream: Optional[torch.cuda.Stream] = None

    @property
    def graph(self) -> Optional[torch.cuda.CUDAGraph]:
        """The first captured graph (None until a capture succeeded)."""
        return next(iter(self.graphs.values()))[0][0] if self.graphs else None

    @property
    def graph_count(self) -> int:
        """Graphs in the first captured chain (1 without split points)."""
        return len(next(iter(self.graphs.values()))[0]) if self.graphs else 0

    def _key(self, ids, tokens):  # (shape, packed-row bucket or None, short_batch)
        if tokens is None or self.bucket is None:
            return tuple(ids.shape), None, False
        B, S = ids.shape[0], ids.shape[1]
        # (batches whose sequences all fit the S <= 128 attention kernels launch fewer kernels)
        return tuple(ids.shape), int(self.bucket(tokens, B, S)), short_batch(tokens, S)

    def __call__(self, ids: torch.Tensor, mask: torch.Tensor, labels: torch.Tensor,
                 tokens: Optional[int] = None) -> torch.Tensor:
        self.calls += 1
        if not self.enabled or self.failed:
            return self.step_fn(ids, mask, labels, tokens)
        key = self._key(ids, tokens)
        hit = self.graphs.get(key)
        prepare = getattr(self.step_fn, "prepare", None)
        if hit is not None:
            if prepare is not None:
                prepare()  # eager state the graph does not refresh itself (the model's weight shadow)
            chain, static, loss = hit
            blk = contiguous_block(ids, mask, labels) if static["flat"] is not None else None
            if blk is not None:
                static["flat"].copy_(blk)
            else:
                static["ids"].copy_(ids)
                static["mask"].copy_(mask)
                static["labels"].copy_(labels)
            for g in chain:
                g.replay()
            return loss
        if self.calls <= self.warmup or len(self.graphs) >= self.max_graphs:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                loss = self.step_fn(ids, mask, labels, tokens)
            torch.cuda.current_stream().wait_stream(s)
            return loss
        # capture (the bucket's own row count stands in for the batch's token count:
        # every device-side quantity is recomputed from the mask on each replay)
        (s_ids, s_mask, s_lab), flat = static_block(ids, mask, labels)
        static = {"ids": s_ids, "mask": s_mask, "labels": s_lab, "flat": flat}
        if prepare is not None:
            prepare()
        chain = [torch.cuda.CUDAGraph()]
        try:
            torch.cuda.synchronize()
            with no_gc():
                if not self.split:
                    with torch.cuda.graph(chain[0]):
                        loss = self.step_fn(static["ids"], static["mask"], static["labels"], key_tokens(key))
                else:
                    loss = self._capture_split(chain, static, key_tokens(key))
        except Exception as e:  # pragma: no cover - capture support varies by op
            self.failed = f"{type(e).__name__}: {e}"
            torch.cuda.synchronize()
            return self.step_fn(ids, mask, labels, tokens)
        self.graphs[key] = (chain, static, loss)
        for g in chain:
            g.replay()
        return loss

    def _capture_split(self, chain, static, tokens):
        """torch.cuda.graph's protocol (side capture stream, one memory pool), with the capture
        cut into a chain at the model's split points (``split_point``)."""
        if self._stream is None:
            self._stream = torch.cuda.Stream()
        cs, pool = self._stream, torch.cuda.graph_pool_handle()
        torch.cuda.empty_cache()
        cs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cs):
            _Capture.active = _Capture(chain, pool, self.split)
            chain[0].capture_begin(pool=pool)
            try:
                loss = self.step_fn(static["ids"], static["mask"], static["labels"], tokens)
            finally:
                _Capture.active = None
                chain[-1].capture_end()
        torch.cuda.current_stream().wait_stream(cs)
        return loss
