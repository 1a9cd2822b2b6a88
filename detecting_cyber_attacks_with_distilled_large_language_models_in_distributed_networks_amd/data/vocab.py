"""Deterministic BERT-style WordPiece vocabulary (30,522 entries).

The reference loads ``DistilBertTokenizer.from_pretrained('./distilbert-base-uncased')``
(client1.py:364).  No pretrained files exist offline, and the model is random-init
anyway (BASELINE.json), so we build a vocabulary with the same size and the same
special-token ids as bert-base-uncased:

  [PAD]=0, [unused0..98]=1..99, [UNK]=100, [CLS]=101, [SEP]=102, [MASK]=103

followed by single characters, the template words of the featuriser, every
number 0..999 as a word piece and as a '##' continuation (so digit strings split
into <=3-digit pieces), and '[unusedN]' filler up to 30,522.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

VOCAB_SIZE = 30522
PAD_ID, UNK_ID, CLS_ID, SEP_ID, MASK_ID = 0, 100, 101, 102, 103

TEMPLATE_WORDS = (
    "destination port is flow duration microseconds total forward packets are backward "
    "length of bytes maximum packet minimum per second the a an and to in for on with by "
    "from at as be this that it or not ddos benign attack traffic network tcp udp http https "
    "dns source ip address protocol rate inf nan e"
).split()


def build_vocab() -> List[str]:
    toks: List[str] = ["[PAD]"] + [f"[unused{i}]" for i in range(99)]
    toks += ["[UNK]", "[CLS]", "[SEP]", "[MASK]"]
    n_unused = 99
    while len(toks) < 999:
        toks.append(f"[unused{n_unused}]")
        n_unused += 1
    chars = [chr(c) for c in range(33, 127) if not ("A" <= chr(c) <= "Z")]
    toks += chars
    seen = set(toks)

    def add(t):
        if t not in seen:
            seen.add(t)
            toks.append(t)

    for w in TEMPLATE_WORDS:
        add(w)
    for i in range(1000):
        add(str(i))
    for i in range(10):
        for j in range(10):
            add(f"{i}{j}")  # leading-zero pairs ('05')
    for i in range(10):
        for j in range(10):
            for k in range(10):
                add(f"{i}{j}{k}")  # leading-zero triples ('007')
    for c in chars:
        add("##" + c)
    for i in range(10):
        for j in range(10):
            for k in range(10):
                add(f"##{i}{j}{k}")
    for i in range(100):
        add(f"##{i:02d}")
    for w in TEMPLATE_WORDS:
        add("##" + w)
    while len(toks) < VOCAB_SIZE:
        add(f"[unused{n_unused}]")
        n_unused += 1
    assert len(toks) == VOCAB_SIZE
    return toks


def write_vocab(path: str) -> str:
    with open(path, "w", encoding="utf-8") as f:
        for t in build_vocab():
            f.write(t + "\n")
    return path


def load_vocab(path: Optional[str] = None) -> Dict[str, int]:
    if path is not None and os.path.isdir(path):
        path = os.path.join(path, "vocab.txt")
    if path is not None and os.path.exists(path):
        with open(path, encoding="utf-8") as f:
            toks = [line.rstrip("\n") for line in f]
    else:
        toks = build_vocab()
    return {t: i for i, t in enumerate(toks)}
