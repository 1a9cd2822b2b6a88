"""Split points of a HIP-graph training-step capture (engine/graph.py GraphedTrainStep): the
model calls ``split_point(block)`` after each block's forward (ops/functional.py LayerFn); inside
a split capture that names the block, the current graph ends and the capture continues into a new
graph of the same memory pool.  Kept free of package imports (the model and the engine both use it).
"""
from __future__ import annotations

import os
from typing import Optional

import torch

# Split points of a training-step capture: the step becomes a chain of graphs ending after these
# blocks' forward (FD_GRAPH_SPLIT, comma-separated block indices; empty = one graph).  A replay
# launches the graphs back to back: the GPU starts on the first short graph while the host is still
# submitting the rest, instead of idling through the whole ~110 us submission of one 73-node graph
# -- which every step after a host synchronisation pays (the first step of a timed window).
GRAPH_SPLIT = tuple(int(v) for v in os.environ.get("FD_GRAPH_SPLIT", "").split(",") if v.strip())


class _Capture:
    """The split capture in progress (one at a time, on the capturing thread's stream)."""
    active: Optional["_Capture"] = None

    def __init__(self, graphs, pool, want):
        self.graphs, self.pool, self.want, self.done = graphs, pool, set(want), set()


def split_point(block: int) -> None:
    """Called by the model after block ``block``'s forward (ops/functional.py LayerFn): inside a
    split capture whose split list names it, end the current graph and capture on into a new one
    that shares its memory pool.  A no-op everywhere else."""
    c = _Capture.active
    if c is None or block not in c.want or block in c.done or not torch.cuda.is_current_stream_capturing():
        return
    c.done.add(block)
    c.graphs[-1].capture_end()
    g = torch.cuda.CUDAGraph()
    g.capture_begin(pool=c.pool)
    c.graphs.append(g)
