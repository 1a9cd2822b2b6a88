"""BERT WordPiece tokenizer (uncased) with a native C++ batch path.

Replaces ``DistilBertTokenizer.from_pretrained('./distilbert-base-uncased')``
(client1.py:364) and its per-sample call in ``__getitem__`` (client1.py:38-45):
  * ``tok(text, add_special_tokens=True, max_length=128, padding='max_length',
    truncation=True, return_tensors='pt')`` returns the same dict shape;
  * ``encode_batch(texts, max_len)`` tokenises a whole split once, thread-parallel
    in C++ (csrc/text/text_native.cpp), into int32 ids + lengths.
The pure-Python implementation below is the executable spec the native one is
tested against.
"""
from __future__ import annotations

import os
import unicodedata
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _text_native
from .vocab import CLS_ID, PAD_ID, SEP_ID, UNK_ID, build_vocab


def _is_punct(ch: str) -> bool:
    cp = ord(ch)
    if 33 <= cp <= 47 or 58 <= cp <= 64 or 91 <= cp <= 96 or 123 <= cp <= 126:
        return True
    return False


def _is_control(ch: str) -> bool:
    if ch in "\t\n\r":
        return False
    cp = ord(ch)
    return cp < 32 or cp == 127 or 0x80 <= cp < 0xA0


class WordPieceTokenizer:
    def __init__(self, vocab: Optional[Sequence[str]] = None, lower: bool = True, max_chars: int = 100,
                 native: Optional[bool] = None):
        self.vocab_list = list(vocab) if vocab is not None else build_vocab()
        self.vocab: Dict[str, int] = {t: i for i, t in enumerate(self.vocab_list)}
        self.lower, self.max_chars = lower, max_chars
        self._native = None
        if native is None or native:
            ext = _text_native.load()
            if ext is None and native:
                raise RuntimeError("native text extension not available")
            if ext is not None:
                self._native = ext.WordPiece(self.vocab_list, lower, max_chars, UNK_ID, CLS_ID, SEP_ID, PAD_ID)

    # ------------------------------------------------------------------ construction
    @classmethod
    def from_pretrained(cls, path: Optional[str] = None, **kw) -> "WordPieceTokenizer":
        if path is not None:
            vf = os.path.join(path, "vocab.txt") if os.path.isdir(path) else path
            if os.path.exists(vf):
                with open(vf, encoding="utf-8") as f:
                    return cls([ln.rstrip("\n") for ln in f], **kw)
        return cls(None, **kw)

    def save_vocabulary(self, path: str) -> str:
        os.makedirs(path, exist_ok=True)
        out = os.path.join(path, "vocab.txt")
        with open(out, "w", encoding="utf-8") as f:
            f.write("\n".join(self.vocab_list) + "\n")
        return out

    @property
    def vocab_size(self) -> int:
        return len(self.vocab_list)

    @property
    def is_native(self) -> bool:
        return self._native is not None

    # ------------------------------------------------------------------ python spec
    def _basic(self, text: str) -> List[str]:
        words, cur = [], []
        for ch in text:
            if ord(ch) == 0 or ord(ch) == 0xFFFD or _is_control(ch):
                continue
            if ch in " \t\n\r":
                if cur:
                    words.append("".join(cur))
                    cur = []
                continue
            if ord(ch) < 128:
                if self.lower:
                    ch = ch.lower()
                if _is_punct(ch):
                    if cur:
                        words.append("".join(cur))
                        cur = []
                    words.append(ch)
                    continue
            cur.append(ch)
        if cur:
            words.append("".join(cur))
        return words

    def _wordpiece(self, word: str) -> List[str]:
        if len(word) > self.max_chars:
            return ["[UNK]"]
        out, start = [], 0
        while start < len(word):
            end, cur = len(word), None
            while start < end:
                sub = word[start:end]
                if start > 0:
                    sub = "##" + sub
                if sub in self.vocab:
                    cur = sub
                    break
                end -= 1
            if cur is None:
                return ["[UNK]"]
            out.append(cur)
            start = end
        return out

    def tokenize(self, text: str) -> List[str]:
        if self._native is not None:
            return self._native.tokenize(text)
        return self.tokenize_py(text)

    def tokenize_py(self, text: str) -> List[str]:
        return [p for w in self._basic(text) for p in self._wordpiece(w)]

    def encode_py(self, text: str, max_len: int) -> List[int]:
        ids = [self.vocab.get(t, UNK_ID) for t in self.tokenize_py(text)][: max_len - 2]
        return [CLS_ID] + ids + [SEP_ID]

    # ------------------------------------------------------------------ batch API
    def encode_batch(self, texts: Sequence[str], max_len: int = 128, threads: int = 8) -> Tuple[np.ndarray, np.ndarray]:
        """-> (ids int32 [N, max_len] padded with [PAD], lengths int32 [N])."""
        texts = [str(t) for t in texts]
        if self._native is not None:
            return self._native.encode_batch(texts, max_len, threads)
        ids = np.zeros((len(texts), max_len), np.int32)
        lens = np.zeros(len(texts), np.int32)
        for i, t in enumerate(texts):
            e = self.encode_py(t, max_len)
            ids[i, :len(e)] = e
            lens[i] = len(e)
        return ids, lens

    def __call__(self, text, add_special_tokens: bool = True, max_length: int = 128, padding="max_length",
                 truncation: bool = True, return_tensors: Optional[str] = None):
        single = isinstance(text, str)
        ids, lens = self.encode_batch([text] if single else list(text), max_length)
        mask = (np.arange(max_length)[None, :] < lens[:, None]).astype(np.int64)
        ids = ids.astype(np.int64)
        if return_tensors == "pt":
            return {"input_ids": torch.from_numpy(ids), "attention_mask": torch.from_numpy(mask)}
        if single:
            return {"input_ids": ids[0].tolist(), "attention_mask": mask[0].tolist()}
        return {"input_ids": ids.tolist(), "attention_mask": mask.tolist()}

    def convert_ids_to_tokens(self, ids):
        return [self.vocab_list[i] for i in ids]


# Alias with the reference's class name (client1.py:5).
DistilBertTokenizer = WordPieceTokenizer
