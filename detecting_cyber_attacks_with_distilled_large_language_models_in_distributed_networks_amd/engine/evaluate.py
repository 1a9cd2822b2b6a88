"""Evaluation (reference ``evaluate_model``, client1.py:118-150).

Returns the reference 8-tuple ``(accuracy %, avg_loss, precision, recall, f1,
confusion_matrix, all_labels, all_probs)`` with identical semantics: accuracy
in percent, ``avg_loss`` = mean of per-batch mean CE (the last, short batch
weighs like a full one), sklearn-binary P/R/F1 (zero_division -> 0), sklearn
confusion-matrix layout.  On GPU the per-batch loss/argmax/confusion counts are
accumulated by one fused kernel into device counters (the reference syncs the
host four times per batch, client1.py:135-142); one sync at the end.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from ..utils.metrics import binary_prf, confusion


@torch.no_grad()
def evaluate_model(model, loader, criterion=None, device=None, log=None, name: str = "Test"):
    if log:
        log.phase("Starting model evaluation")
    was_training = model.training
    model.eval()
    dev = model.device
    n = loader.n if hasattr(loader, "n") else len(loader.dataset)
    probs = torch.empty(n, dtype=torch.float32, device=dev)
    preds = torch.empty(n, dtype=torch.int64, device=dev)
    labels_all = torch.empty(n, dtype=torch.int64, device=dev)
    nb = 0
    off = 0
    if dev.type == "cuda":
        from ..ops import kernels as K
        acc = torch.zeros(1, dtype=torch.float64, device=dev)
        counts = torch.zeros(5, dtype=torch.int64, device=dev)
        packed = getattr(model, "impl", None) == "hip"
        fwd = None
        if packed:  # unpadded HIP forward replayed from graphs (cached on the model across evals)
            from .infer import GraphedForward
            fwd = getattr(model, "_graphed_eval", None)
            if fwd is None or fwd.model is not model:
                fwd = GraphedForward(model)
                model._graphed_eval = fwd
        for batch in loader:
            if fwd is not None and batch.get("n_tokens") is not None:
                logits = fwd(batch["input_ids"], batch["attention_mask"], batch["n_tokens"])
            else:
                logits = model(batch["input_ids"], batch["attention_mask"])
            b = logits.shape[0]
            lab = batch["labels"]
            K.eval_metrics(logits, lab, acc, counts, probs[off:off + b], preds[off:off + b])
            labels_all[off:off + b] = lab
            off += b
            nb += 1
        loss_sum = acc.item()
        correct, tp, fp, fn, tn = counts.tolist()
        if packed and getattr(model, "fuse_ln", False):
            K.check_ln_error(dev, model.config.dim)  # a timed-out LayerNorm rendezvous is fatal
    else:
        loss_sum = 0.0
        correct = tp = fp = fn = tn = 0
        for batch in loader:
            logits = model(batch["input_ids"], batch["attention_mask"]).float()
            lab = batch["labels"]
            b = logits.shape[0]
            loss_sum += torch.nn.functional.cross_entropy(logits, lab).item()
            pr = torch.softmax(logits, dim=1)[:, 1]
            pd = (logits[:, 1] > logits[:, 0]).long()
            probs[off:off + b] = pr
            preds[off:off + b] = pd
            labels_all[off:off + b] = lab
            correct += int((pd == lab).sum())
            tp += int(((pd == 1) & (lab == 1)).sum())
            fp += int(((pd == 1) & (lab == 0)).sum())
            fn += int(((pd == 0) & (lab == 1)).sum())
            tn += int(((pd == 0) & (lab == 0)).sum())
            off += b
            nb += 1
    total = off
    accuracy = 100.0 * correct / max(total, 1)
    avg_loss = loss_sum / max(nb, 1)
    precision, recall, f1 = binary_prf(tp, fp, fn)
    all_labels = labels_all[:total].cpu().numpy().tolist()
    all_preds = preds[:total].cpu().numpy().tolist()
    cm = confusion(tn, fp, fn, tp, set(all_labels) | set(all_preds))
    all_probs = probs[:total].cpu().numpy().tolist()
    if log:
        log.info(f"{name} Accuracy: {accuracy:.2f}%, Loss: {avg_loss:.4f}, Precision: {precision:.4f}, "
                 f"Recall: {recall:.4f}, F1-Score: {f1:.4f}", accuracy=accuracy, loss=avg_loss,
                 precision=precision, recall=recall, f1=f1)
        log.phase("Finished model evaluation")
    if was_training:
        model.train()
    return accuracy, avg_loss, precision, recall, f1, cm, all_labels, all_probs
