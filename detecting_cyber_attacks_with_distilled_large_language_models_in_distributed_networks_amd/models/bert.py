"""BERT-base teacher for knowledge distillation (BASELINE.json config 5).

The reference has no teacher ("Distilled" in its title refers to DistilBERT;
SURVEY 7.0).  The extension trains / loads a 12-layer BERT-base classifier and
distils it into the 6-layer DistilBERT ``DDoSClassifier`` (soft targets at
temperature T + hard-label CE).

Architecture = the DistilBERT block stack with BERT-base hyper-parameters
(12 x [post-LN MHSA(12 heads) + GELU FFN 3072], hidden 768) plus BERT's
token-type embedding, so every hot op runs on the same gfx950 kernels (the
type-0 row is folded into the position table each forward: token_type_ids are
all zero for single-sentence classification; the table is an arena parameter and
trains on the HIP path through the position gradient).  Parameters live in their own
arena under the ``bert.`` prefix; ``load_hf_bert`` maps HuggingFace
``BertForSequenceClassification`` keys when a checkpoint is available offline.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn as nn

from .distilbert import DDoSClassifier, DistilBertConfig, _P


def bert_base_config(**kw) -> DistilBertConfig:
    cfg = DistilBertConfig(n_layers=12, n_heads=12, dim=768, hidden_dim=3072)
    for k, v in kw.items():
        setattr(cfg, k, v)
    return cfg


class BertTeacherClassifier(DDoSClassifier):
    """12-layer BERT-base + Dropout + Linear(768, 2) on the shared kernel path.

    The token-type table lives in the parameter arena (``TOKEN_TYPES = 2``), so the
    optimizer, FedAvg and checkpoints treat it like every other parameter; with
    token_type_ids all 0 its row 0 is folded into the position table the kernels read and
    its gradient is the column sum of the position gradient (ops/functional.py
    EmbeddingFn) -- it trains on the HIP path too."""

    PREFIX = "bert."
    TOKEN_TYPES = 2

    def __init__(self, local_model_path: Optional[str] = None, config: Optional[DistilBertConfig] = None,
                 device=None, impl: str = "auto", seed: int = 1, head_dropout: float = 0.1):
        cfg = config or bert_base_config()
        super().__init__(None, config=cfg, device="cpu", impl=impl, seed=seed, head_dropout=head_dropout)
        if local_model_path and os.path.isdir(local_model_path):
            load_hf_bert(self, local_model_path)
        self.to(device or "cpu")

    def state_dict(self, *args, **kwargs):
        sd = super().state_dict(*args, **kwargs)
        out = type(sd)()
        for k, v in sd.items():
            out[self.PREFIX + k[len("distilbert."):] if k.startswith("distilbert.") else k] = v
        return out

    def load_state_dict(self, sd, strict: bool = True, assign: bool = False):
        mapped = type(sd)() if hasattr(sd, "keys") else {}
        for k, v in sd.items():
            mapped["distilbert." + k[len(self.PREFIX):] if k.startswith(self.PREFIX) else k] = v
        return super().load_state_dict(mapped, strict=strict, assign=assign)


_HF_LAYER_MAP = {
    "attention.self.query": "attention.q_lin", "attention.self.key": "attention.k_lin",
    "attention.self.value": "attention.v_lin", "attention.output.dense": "attention.out_lin",
    "attention.output.LayerNorm": "sa_layer_norm", "intermediate.dense": "ffn.lin1",
    "output.dense": "ffn.lin2", "output.LayerNorm": "output_layer_norm",
}


def load_hf_bert(model: BertTeacherClassifier, path: str) -> int:
    """Map HF BertForSequenceClassification weights (safetensors / weights_only .bin)."""
    sd = None
    st, pt = os.path.join(path, "model.safetensors"), os.path.join(path, "pytorch_model.bin")
    if os.path.exists(st):
        from safetensors.torch import load_file
        sd = load_file(st)
    elif os.path.exists(pt):
        sd = torch.load(pt, map_location="cpu", weights_only=True)
    if sd is None:
        return 0
    n = 0
    A = model.arena
    for k, v in sd.items():
        k2 = k.removeprefix("bert.")
        tgt = None
        if k2.startswith("embeddings."):
            tgt = "distilbert." + k2
        elif k2.startswith("encoder.layer."):
            parts = k2.split(".")
            i, rest = parts[2], ".".join(parts[3:])
            for src, dst in _HF_LAYER_MAP.items():
                if rest.startswith(src + "."):
                    tgt = f"distilbert.transformer.layer.{i}.{dst}.{rest[len(src) + 1:]}"
                    tgt = tgt.replace(".gamma", ".weight").replace(".beta", ".bias")
                    break
        elif k2.startswith("classifier."):
            tgt = k2
        if tgt and tgt in A.offsets and tuple(v.shape) == A.offsets[tgt][1]:
            A.view(tgt).copy_(v.float())
            n += 1
    return n


def kd_loss(student_logits: torch.Tensor, teacher_logits: torch.Tensor, labels: torch.Tensor,
            temperature: float = 2.0, alpha: float = 0.5) -> torch.Tensor:
    """alpha * CE(student, y) + (1 - alpha) * T^2 * KL(softmax(t/T) || softmax(s/T))."""
    T = temperature
    hard = torch.nn.functional.cross_entropy(student_logits, labels)
    soft = torch.nn.functional.kl_div(torch.log_softmax(student_logits / T, dim=-1),
                                      torch.log_softmax(teacher_logits.detach() / T, dim=-1),
                                      reduction="batchmean", log_target=True) * (T * T)
    return alpha * hard + (1.0 - alpha) * soft
