"""Failure detection for the federated job: heartbeats + a health-checked barrier.

Reference behaviour: every socket has a 300 s timeout; a client
that dies leaves the server blocked in ``accept`` until that timeout raises
(server.py:119,126) and the other client retrying ``wait_for_server`` five
times (client1.py:298-336).  A dead peer is indistinguishable from a slow one.

Here each rank runs a heartbeat thread that bumps a counter in the job's
TCPStore (torch.distributed's rendezvous store) every ``interval`` seconds.
Before a collective that every client must join (the FedAvg all-reduce),
ranks meet in ``HealthMonitor.barrier``: a store-counter barrier that, while
it waits, watches every peer's heartbeat counter.  A peer whose counter has
not moved for ``stale_s`` seconds (measured on the local clock, so host clock
skew does not matter) is declared dead and the barrier raises ``PeerFailure``
naming it -- within seconds, instead of hanging in RCCL until the collective
timeout.  A slow-but-alive peer (still training) keeps beating and is waited
for up to ``timeout``.

Elastic recovery: the raised error ends the rank with a non-zero exit; under
``torchrun --max-restarts N`` (``cli launch --max-restarts N``) the agent
restarts the whole group, every client reloads its round checkpoint
(``clientN_model.pth`` + ``clientN_fed_state.json``) and the job continues at
the first unfinished round.  Store keys carry the restart count, so a
restarted group never sees the previous attempt's barrier arrivals.
"""
from __future__ import annotations

import os
import threading
import time
from typing import Dict, List, Optional

import torch.distributed as dist


class PeerFailure(RuntimeError):
    def __init__(self, dead: List[int], where: str):
        super().__init__(f"peer rank(s) {dead} stopped heartbeating ({where})")
        self.dead = dead


def _open_store(timeout_s: float):
    """A client connection of our own to the job's TCPStore (the heartbeat thread must
    not share the main thread's connection)."""
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("MASTER_PORT", "29500"))
    import datetime
    return dist.TCPStore(host, port, is_master=False, timeout=datetime.timedelta(seconds=timeout_s),
                         wait_for_workers=False)


class HealthMonitor:
    def __init__(self, rank: int, world: int, interval: float = 1.0, stale_s: float = 10.0,
                 timeout_s: float = 300.0, store=None):
        self.rank, self.world = rank, world
        self.interval, self.stale_s, self.timeout_s = interval, stale_s, timeout_s
        gen = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
        self.prefix = f"fedddos/{gen}/"
        self._store = store or _open_store(timeout_s)
        self._beat_store = store or _open_store(timeout_s)
        self._stop = threading.Event()
        self._seen: Dict[int, tuple] = {}
        self._lock = threading.Lock()
        self._thread = threading.Thread(target=self._run, name="fedddos-heartbeat", daemon=True)
        self._beat()
        self._thread.start()

    # ---------------------------------------------------------------- heartbeat
    def _beat(self):
        with self._lock:
            self._beat_store.add(f"{self.prefix}hb/{self.rank}", 1)

    def _run(self):
        while not self._stop.wait(self.interval):
            try:
                self._beat()
            except Exception:  # store gone (rank 0 / agent died): the main thread finds out
                return

    def stop(self):
        self._stop.set()

    # ---------------------------------------------------------------- detection
    def dead_peers(self) -> List[int]:
        """Ranks whose heartbeat counter has not moved for ``stale_s`` (local clock)."""
        now = time.monotonic()
        dead = []
        for r in range(self.world):
            if r == self.rank:
                continue
            v = int(self._store.add(f"{self.prefix}hb/{r}", 0))
            last = self._seen.get(r)
            if last is None or last[0] != v:
                self._seen[r] = (v, now)
            elif now - last[1] > self.stale_s:
                dead.append(r)
        return dead

    def barrier(self, name: str, timeout_s: Optional[float] = None):
        """All ranks arrive, or raise PeerFailure (a peer died) / TimeoutError (alive but late)."""
        key = f"{self.prefix}bar/{name}"
        self._store.add(key, 1)
        t0 = time.monotonic()
        limit = self.timeout_s if timeout_s is None else timeout_s
        poll = min(0.05, self.interval)
        while int(self._store.add(key, 0)) < self.world:
            dead = self.dead_peers()
            if dead:
                raise PeerFailure(dead, f"barrier {name!r}")
            if time.monotonic() - t0 > limit:
                raise TimeoutError(f"barrier {name!r}: peers alive but not arrived after {limit:.0f} s")
            time.sleep(poll)
            poll = min(poll * 2, self.interval)


_MON: Optional[HealthMonitor] = None


def start(interval: float = 1.0, stale_s: float = 10.0, timeout_s: float = 300.0) -> Optional[HealthMonitor]:
    """Start this rank's heartbeat (no-op for a single process)."""
    global _MON
    if _MON is None and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        _MON = HealthMonitor(dist.get_rank(), dist.get_world_size(), interval, stale_s, timeout_s)
    return _MON


def monitor() -> Optional[HealthMonitor]:
    return _MON


def stop():
    global _MON
    if _MON is not None:
        _MON.stop()
    _MON = None
