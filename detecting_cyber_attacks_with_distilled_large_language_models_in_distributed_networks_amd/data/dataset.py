"""Pre-tokenised CICIDS2017 text dataset + device-resident batch loader.

``CICIDS2017Dataset(texts, labels, tokenizer, max_len=128)`` keeps the
reference's constructor and ``__getitem__`` contract (client1.py:26-50:
``{'input_ids', 'attention_mask', 'labels'}``) but tokenises the whole split
ONCE in C++ at construction instead of on every access of every epoch.

``DeviceLoader`` replaces ``DataLoader(bs=16, shuffle=...)`` (client1.py:370-372):
the split lives on the GPU (13.5k x 128 int64 ids = 14 MB), each epoch draws a
device permutation and batches are index-gathers -- no host work, no H2D copy
and no sync per step.  ``drop_last=False`` like the reference.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .tokenizer import WordPieceTokenizer


class CICIDS2017Dataset(torch.utils.data.Dataset):
    def __init__(self, texts: Sequence[str], labels: Sequence[int], tokenizer: Optional[WordPieceTokenizer] = None,
                 max_len: int = 128, ids: Optional[np.ndarray] = None, lengths: Optional[np.ndarray] = None):
        self.max_len = max_len
        self.labels = torch.as_tensor(np.asarray(labels, dtype=np.int64))
        if ids is None:
            tokenizer = tokenizer or WordPieceTokenizer()
            ids, lengths = tokenizer.encode_batch(list(texts), max_len)
        self.texts = texts
        self.input_ids = torch.from_numpy(np.ascontiguousarray(ids).astype(np.int64))
        lengths = torch.from_numpy(np.asarray(lengths).astype(np.int64))
        self.attention_mask = (torch.arange(max_len)[None, :] < lengths[:, None]).to(torch.int64)

    def __len__(self) -> int:
        return len(self.labels)

    def __getitem__(self, idx) -> Dict[str, torch.Tensor]:
        return {"input_ids": self.input_ids[idx], "attention_mask": self.attention_mask[idx],
                "labels": self.labels[idx]}


class PackedTokens(int):
    """A batch's real-token count (an ``int`` everywhere it is used as one) that also carries the
    batch's longest sequence, ``max_len`` -- both known on the host without a device sync.  The
    model's packed path at S > 128 runs the S <= 128 attention kernels alone when max_len <= 128
    (ops/kernels.py attn_fwd ``short``); graph keys separate such batches (``short_batch``)."""

    def __new__(cls, total: int, max_len: int):
        obj = super().__new__(cls, int(total))
        obj.max_len = int(max_len)
        return obj

    def __reduce__(self):
        return (PackedTokens, (int(self), self.max_len))


_SHORT = os.environ.get("FD_ATTN_SHORT", "1") != "0"  # 0: never (the length split alone decides)


def short_batch(tokens, S: int) -> bool:
    """Every sequence of the batch has <= 128 real tokens while the padded length S is longer."""
    return _SHORT and S > 128 and 0 < getattr(tokens, "max_len", 0) <= 128


class DeviceLoader:
    """Iterates {'input_ids','attention_mask','labels'} device batches."""

    def __init__(self, dataset: CICIDS2017Dataset, batch_size: int = 16, shuffle: bool = False,
                 device="cpu", seed: int = 0, drop_last: bool = False):
        self.device = torch.device(device)
        self.ids = dataset.input_ids.to(self.device)
        self.mask = dataset.attention_mask.to(self.device)
        self.labels = dataset.labels.to(self.device)
        self.n = len(dataset)
        # host copy of the per-row real-token counts: every batch carries ``n_tokens`` (a
        # Python int, no device sync) for the model's unpadded path
        self.lengths = dataset.attention_mask.detach().to("cpu").sum(1).to(torch.int64)
        self.batch_size, self.shuffle, self.drop_last = batch_size, shuffle, drop_last
        self.gen = torch.Generator(device="cpu").manual_seed(seed)
        self.epoch = 0

    def __len__(self) -> int:
        if self.drop_last:
            return self.n // self.batch_size
        return (self.n + self.batch_size - 1) // self.batch_size

    def _epoch_blocks(self, perm: Optional[torch.Tensor], nfull: int) -> Optional[torch.Tensor]:
        """The epoch's full batches gathered once into one buffer, batch i = row i laid out as
        ids | mask | labels back to back: a step reads three contiguous views of one block
        (one gather per epoch instead of three per step, and a graph replay refreshes its
        inputs with one copy).  None when the dtypes differ."""
        if nfull == 0 or not (self.ids.dtype == self.mask.dtype == self.labels.dtype):
            return None
        B, S = self.batch_size, self.ids.shape[1]
        rows = nfull * B
        sel = (lambda t: t.index_select(0, perm[:rows])) if perm is not None else (lambda t: t[:rows])
        blk = torch.empty(nfull, B * (2 * S + 1), dtype=self.ids.dtype, device=self.device)
        blk[:, :B * S].copy_(sel(self.ids).reshape(nfull, B * S))
        blk[:, B * S:2 * B * S].copy_(sel(self.mask).reshape(nfull, B * S))
        blk[:, 2 * B * S:].copy_(sel(self.labels).reshape(nfull, B))
        return blk

    def __iter__(self):
        if self.shuffle:
            perm_cpu = torch.randperm(self.n, generator=self.gen)
            perm = perm_cpu.to(self.device)
        else:
            perm_cpu = perm = None
        self.epoch += 1
        B, S = self.batch_size, self.ids.shape[1]
        nfull = self.n // B
        blocks = self._epoch_blocks(perm, nfull) if self.ids.dim() == 2 else None
        for i in range(len(self)):
            if blocks is not None and i < nfull:
                row = blocks[i]
                lo, hi = i * B, (i + 1) * B
                lens = self.lengths[perm_cpu[lo:hi]] if perm_cpu is not None else self.lengths[lo:hi]
                yield {"input_ids": row[:B * S].view(B, S), "attention_mask": row[B * S:2 * B * S].view(B, S),
                       "labels": row[2 * B * S:], "n_tokens": PackedTokens(lens.sum(), lens.max())}
                continue
            lo, hi = i * self.batch_size, min(self.n, (i + 1) * self.batch_size)
            if perm is None:
                lens = self.lengths[lo:hi]
                yield {"input_ids": self.ids[lo:hi], "attention_mask": self.mask[lo:hi], "labels": self.labels[lo:hi],
                       "n_tokens": PackedTokens(lens.sum(), lens.max())}
            else:
                idx = perm[lo:hi]
                yield {"input_ids": self.ids.index_select(0, idx), "attention_mask": self.mask.index_select(0, idx),
                       "labels": self.labels.index_select(0, idx),
                       "n_tokens": PackedTokens(self.lengths[perm_cpu[lo:hi]].sum(), self.lengths[perm_cpu[lo:hi]].max())}


@dataclass
class ClientData:
    train: CICIDS2017Dataset
    val: CICIDS2017Dataset
    test: CICIDS2017Dataset
    n_rows: int


def build_client_data(frame, client_id: int, data_fraction: float = 0.1, base_seed: int = 42, max_len: int = 128,
                      tokenizer: Optional[WordPieceTokenizer] = None, partition: str = "iid_overlap",
                      num_clients: int = 1, log=None) -> ClientData:
    """Client k's 60/20/20 splits (client1.py:363-369 with seed 42 + k).

    ``iid_overlap`` (reference): each client samples ``data_fraction`` of the full
    frame independently with its own seed -> ~10 % row overlap between clients.
    ``disjoint``: rows are first dealt round-robin to clients by a seed-0 permutation.
    """
    from .featurize import clean_frame, render_texts, split_60_20_20
    seed = base_seed + client_id
    if log:
        log("Starting data preprocessing")
    df = clean_frame(frame) if isinstance(frame, __import__("pandas").DataFrame) else frame
    if partition == "disjoint" and num_clients > 1:
        order = np.random.default_rng(0).permutation(len(df))
        df = df.iloc[order[client_id::num_clients]]
        frac = min(1.0, data_fraction * num_clients)
    else:
        frac = data_fraction
    df = df.sample(frac=frac, random_state=seed)
    texts = render_texts(df)
    labels = (df["Label"].to_numpy() == "DDoS").astype(np.int64).tolist()
    if log:
        log("Finished data preprocessing")
    (xtr, ytr), (xva, yva), (xte, yte) = split_60_20_20(texts, labels, seed)
    tok = tokenizer or WordPieceTokenizer()
    return ClientData(CICIDS2017Dataset(xtr, ytr, tok, max_len), CICIDS2017Dataset(xva, yva, tok, max_len),
                      CICIDS2017Dataset(xte, yte, tok, max_len), len(df))
