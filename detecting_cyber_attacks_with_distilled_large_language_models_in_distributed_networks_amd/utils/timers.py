"""Per-phase wall timers (the reference only has datetime stamps) and
HIP-event step timers; optional torch.profiler trace and a rocprofv3 command helper."""
from __future__ import annotations

import contextlib
import time
from collections import defaultdict
from typing import Dict, List, Optional

import torch


class PhaseTimer:
    """Accumulates wall time per named phase (preprocess, train, eval, fedavg, plot, ...)."""

    def __init__(self, sync_cuda: bool = True):
        self.totals: Dict[str, float] = defaultdict(float)
        self.counts: Dict[str, int] = defaultdict(int)
        self.sync = sync_cuda and torch.cuda.is_available()

    @contextlib.contextmanager
    def __call__(self, name: str):
        if self.sync:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        try:
            yield
        finally:
            if self.sync:
                torch.cuda.synchronize()
            self.totals[name] += time.perf_counter() - t0
            self.counts[name] += 1

    def summary(self) -> Dict[str, float]:
        return {k: round(v, 6) for k, v in self.totals.items()}


class StepTimer:
    """HIP-event timing of GPU work between start() and stop() without host syncs in between."""

    def __init__(self):
        self.events: List = []

    def start(self):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self.events.append([e, None])

    def stop(self):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self.events[-1][1] = e

    def millis(self) -> List[float]:
        torch.cuda.synchronize()
        return [a.elapsed_time(b) for a, b in self.events if b is not None]


@contextlib.contextmanager
def torch_trace(path: Optional[str]):
    """Optional torch.profiler chrome trace of a region."""
    if not path:
        yield None
        return
    from torch.profiler import ProfilerActivity, profile
    acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if torch.cuda.is_available() else [])
    with profile(activities=acts) as prof:
        yield prof
    prof.export_chrome_trace(path)


def rocprof_cmd(out_dir: str, argv: List[str], pmc: Optional[List[str]] = None) -> List[str]:
    """rocprofv3 command line (kernel trace + stats, or a separate PMC pass)."""
    cmd = ["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", out_dir]
    if pmc:
        cmd += ["--pmc"] + pmc
    return cmd + ["--"] + argv
