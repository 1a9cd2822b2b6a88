"""Intra-client data parallelism: one federated client spread over k GPUs.

The reference has one process per client and no per-step gradient exchange
("Data parallel ... No"); BASELINE.json's north star asks for each
client to run *local data-parallel training*.  Here a job of W = C * k ranks
is C federated clients of k GPUs each:

  rank r -> client r // k, data-parallel replica r % k

* Every replica of a client holds identical weights (rank-0 broadcast at the
  start, identical Adam updates after), walks the client's shuffled batches in
  the same order and takes its ``tensor_split`` share of each batch.
* Gradients are summed over the client's k replicas on a per-client process
  group (RCCL over xGMI on GPUs, gloo on CPU).  The loss is pre-scaled by the
  replica's share of the client batch (n_r / n), so the SUM is exactly the
  gradient of the client-batch mean -- the same optimisation problem as one GPU
  at the same ``batch_size``.
* HIP path: each transformer block's gradient span (7.1 M fp32, 28 MB) is
  launched as an async all-reduce from the backward hook the moment the block's
  gradients are final, so the exchange of block i overlaps the backward GEMMs of
  blocks i-1..0; ``finish()`` adds the embedding/head bucket and waits.
* The word-embedding gradient is sparse (only rows of ids in the batch carry a
  value, ``model.emb_now``): instead of all-reducing the 94 MB table the
  replicas OR their row flags (30 K ints), compact the union of rows with
  ``nonzero_static`` (fixed size -> no host sync), all-reduce only those rows
  (<= one row per token of the client batch) and scatter them back.
* FedAvg across clients stays ONE all-reduce over the whole world: replicas of
  a client are identical, so giving each weight w/k yields the client average.
* With a framework communicator over the client's group (``NativeComm(group=...)``, RCCL) every
  collective of the exchange is issued on a side stream forked from the compute stream and joined
  back in ``finish()`` -- nothing synchronises the host -- so the whole data-parallel step (forward,
  backward with the overlapped block all-reduces, the sparse row exchange, Adam) is captured into
  ONE HIP graph (``capturable``); torch.distributed's work objects are not capturable, so without
  it the step stays eager.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


@dataclass
class ClientTopology:
    world_size: int = 1
    rank: int = 0
    gpus_per_client: int = 1
    dp_group: Optional[object] = None

    @property
    def num_clients(self) -> int:
        return self.world_size // self.gpus_per_client

    @property
    def client_idx(self) -> int:
        return self.rank // self.gpus_per_client

    @property
    def dp_rank(self) -> int:
        return self.rank % self.gpus_per_client

    @property
    def dp(self) -> bool:
        return self.gpus_per_client > 1

    def client_ranks(self, c: int) -> List[int]:
        k = self.gpus_per_client
        return list(range(c * k, (c + 1) * k))


def make_topology(gpus_per_client: int = 1) -> ClientTopology:
    """Split the world into clients of ``gpus_per_client`` consecutive ranks.

    Every rank creates every per-client group (torch.distributed requires
    ``new_group`` to be called collectively, in the same order)."""
    on = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size() if on else 1
    rank = dist.get_rank() if on else 0
    k = max(1, int(gpus_per_client))
    if world % k:
        raise ValueError(f"world size {world} is not a multiple of gpus_per_client={k}")
    topo = ClientTopology(world, rank, k, None)
    if k > 1:
        for c in range(world // k):
            g = dist.new_group(topo.client_ranks(c))
            if c == topo.client_idx:
                topo.dp_group = g
    return topo


class DPShardLoader:
    """This replica's share of each client batch (replicas iterate the same shuffled order).

    Yields the usual batch dict plus ``loss_scale`` = n_r / n.  A final batch with fewer
    rows than replicas is skipped (every replica must contribute to each exchange)."""

    def __init__(self, loader, dp_rank: int, k: int):
        self.loader, self.dp_rank, self.k = loader, dp_rank, k

    def __len__(self) -> int:
        n, bs = self.loader.n, self.loader.batch_size
        full = n // bs
        rest = n - full * bs
        if self.loader.drop_last or rest == 0:
            return full
        return full + (1 if rest >= self.k else 0)

    def __iter__(self):
        for b in self.loader:
            n = b["labels"].shape[0]
            if n < self.k:
                continue
            parts = {key: torch.tensor_split(v, self.k)[self.dp_rank] for key, v in b.items() if torch.is_tensor(v)}
            parts["loss_scale"] = parts["labels"].shape[0] / n
            yield parts


class GradSync:
    """Sum a client's gradients over its k data-parallel replicas (see module doc)."""

    def __init__(self, model, group, k: int, max_rows: Optional[int] = None, overlap: bool = True,
                 ncomm=None):
        self.model, self.group, self.k = model, group, k
        self.overlap = overlap
        self.arena = model.arena
        V = model.config.vocab_size
        self.max_rows = int(min(V, max_rows or V))
        self.works: List = []
        self.done: List[Tuple[int, int]] = []
        self.loss_scale = torch.ones((), dtype=torch.float32, device=self.arena.device)
        # ncomm: NativeComm over this client's group -> stream-ordered, graph-capturable exchange
        self.ncomm = ncomm if (ncomm is not None and self.arena.device.type == "cuda") else None
        self.side = torch.cuda.Stream(device=self.arena.device) if self.ncomm is not None else None
        self._forked = False
        self._prev_hook = model.layer_grads_hook
        if overlap:
            model.layer_grads_hook = self._on_layer
            # collectives now run beside the backward: the model keeps its LayerNorm-fused backward
            # GEMMs off (their row-block rendezvous needs every tile resident; ops/kernels.py ln_fusable)
            model.collectives_in_backward = True

    @property
    def capturable(self) -> bool:
        """Whether a step using this exchange may be captured into a HIP graph."""
        return self.ncomm is not None

    # -------------------------------------------------------------- pieces
    def _fork(self):
        """Side stream waits for everything the compute stream issued so far (the gradients the
        next collective reads are final in stream order)."""
        self.side.wait_stream(torch.cuda.current_stream(self.arena.device))
        self._forked = True

    def _allreduce(self, t: torch.Tensor, op=None):
        if self.ncomm is not None:
            self._fork()
            with torch.cuda.stream(self.side):
                self.ncomm.all_reduce_(t, "max" if op == dist.ReduceOp.MAX else "sum", wait=False)
            return
        w = dist.all_reduce(t, op=op or dist.ReduceOp.SUM, group=self.group, async_op=True)
        self.works.append(w)

    def _on_layer(self, i: int):
        if self._prev_hook is not None:
            raise RuntimeError("GradSync cannot share the backward hook (use ArenaAdam(overlap=False))")
        if not self.model.training:
            return
        off, n = self.model.layer_span(i)
        self._allreduce(self.arena.grad[off:off + n])
        self.done.append((off, n))

    def _sparse_word(self) -> bool:
        m = self.model
        return (getattr(m, "impl", "torch") == "hip" and getattr(m, "sparse_word_grad", False)
                and getattr(m, "emb_now", None) is not None)

    def _word_rows(self):
        """All-reduce only the union of word-embedding rows any replica touched."""
        m = self.model
        woff, V, D = m.word_embedding_span()
        g = self.arena.grad[woff:woff + V * D].view(V, D)
        now = m.emb_now
        native = self.ncomm is not None
        if native:  # the whole exchange on the side stream, after everything computed so far
            self._fork()
        import contextlib
        with torch.cuda.stream(self.side) if native else contextlib.nullcontext():
            union = now.to(torch.int32)
            if native:
                self.ncomm.all_reduce_(union, "max", wait=False)
            else:
                dist.all_reduce(union, op=dist.ReduceOp.MAX, group=self.group)
            rows = torch.nonzero_static(union, size=self.max_rows, fill_value=-1).squeeze(1)
            # filler slots repeat the first real row (the [CLS] id is always present), so the
            # duplicate index_copy_ writes below all carry the same, correct value
            rows = torch.where(rows >= 0, rows, rows[:1])
            keep = now.index_select(0, rows).to(g.dtype)
            buf = g.index_select(0, rows) * keep[:, None]  # zero where only another replica has the row
            if native:
                self.ncomm.all_reduce_(buf, "sum", wait=False)
            else:
                dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group)
            g.index_copy_(0, rows, buf)
            now.copy_(union.clamp_(max=1).to(now.dtype))
            m.emb_ever.bitwise_or_(now)

    # -------------------------------------------------------------- step API
    def set_loss_scale(self, s: float):
        self.loss_scale.fill_(float(s))

    def finish(self):
        """After backward: exchange every span the hooks did not cover, then wait."""
        A = self.arena
        skip = []
        sparse = self._sparse_word()
        if sparse:
            woff, V, D = self.model.word_embedding_span()
            skip.append((woff, V * D))
        covered = sorted(self.done + skip)
        pos = 0
        for off, n in covered:
            if off > pos:
                self._allreduce(A.grad[pos:off])
            pos = max(pos, off + n)
        if pos < A.numel:
            self._allreduce(A.grad[pos:A.numel])
        if sparse:
            self._word_rows()
        for w in self.works:
            w.wait()
        if self.ncomm is not None and self._forked:
            # join: Adam (next on the compute stream) reads the summed gradients; no host sync --
            # an RCCL-reported failure still surfaces here (async error poll, outside capture)
            torch.cuda.current_stream(self.arena.device).wait_stream(self.side)
            self._forked = False
            if not torch.cuda.is_current_stream_capturing():
                self.ncomm.check()
        self.works, self.done = [], []

    def detach(self):
        if self.overlap and self.model.layer_grads_hook == self._on_layer:
            self.model.layer_grads_hook = self._prev_hook
            self.model.collectives_in_backward = False


def make_dp_step_fn(model, optimizer, sync: GradSync, teacher=None, temperature: float = 2.0,
                    alpha: float = 0.5):
    """Data-parallel train step: scaled local loss -> backward (overlapped block
    all-reduces) -> finish the exchange -> Adam.  Returns this replica's share of
    the client-batch mean loss (sum over replicas = the client-batch mean).

    teacher: distillation (engine/train.py make_kd_step_fn) on the replica's shard -- the
    frozen teacher is identical on every replica, so the shard-mean KD losses, scaled by
    the shard shares, sum to the client-batch KD loss exactly as the CE loss does."""
    if getattr(optimizer, "overlap", False):
        raise ValueError("data-parallel clients need ArenaAdam(overlap=False)")
    def step(ids, mask, labels, tokens=None):  # shards run the padded path (no per-shard token count)
        optimizer.zero_grad()
        if teacher is None:
            loss, _ = model.forward_loss(ids, mask, labels)
        else:
            with torch.no_grad():
                t_logits = teacher(ids, mask)
            loss, _ = model.forward_loss(ids, mask, labels, kd=(t_logits, temperature, alpha))
        scaled = loss * sync.loss_scale
        scaled.backward()
        sync.finish()
        optimizer.step()
        return scaled.detach()

    step.prepare = getattr(model, "prepare_replay", None)
    return step


def dp_seed_offset(model, dp_rank: int):
    """Distinct dropout streams per replica (the masks are counter-based on ``model.rng``)."""
    if dp_rank and getattr(model, "rng", None) is not None:
        model.rng.fill_(int(dp_rank) << 20)
    if dp_rank and hasattr(model, "torch_counter"):
        model.torch_counter = int(dp_rank) << 20
