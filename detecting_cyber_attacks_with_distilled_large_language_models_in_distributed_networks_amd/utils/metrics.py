"""Metric tuple helpers + CSV writer with the reference schema.

``evaluate_model`` returns the reference 8-tuple (client1.py:150):
``(accuracy_percent, avg_loss, precision, recall, f1, confusion_matrix, labels, probs)``.
``save_metrics`` writes the 1-row CSV ``Accuracy,Loss,Precision,Recall,F1-Score``
(client1.py:339-350; accuracy in percent, the rest fractions).
"""
from __future__ import annotations

import csv
import os
from typing import Sequence, Tuple

import numpy as np


def binary_prf(tp: int, fp: int, fn: int) -> Tuple[float, float, float]:
    """sklearn precision_recall_fscore_support(average='binary') with zero_division -> 0."""
    p = tp / (tp + fp) if (tp + fp) > 0 else 0.0
    r = tp / (tp + fn) if (tp + fn) > 0 else 0.0
    f = 2 * p * r / (p + r) if (p + r) > 0 else 0.0
    return float(p), float(r), float(f)


def confusion(tn: int, fp: int, fn: int, tp: int, labels_present: Sequence[int]) -> np.ndarray:
    """sklearn confusion_matrix layout [[TN, FP], [FN, TP]]; 1x1 when only one class occurs."""
    present = sorted(set(labels_present))
    if present == [0]:
        return np.array([[tn]], dtype=np.int64)
    if present == [1]:
        return np.array([[tp]], dtype=np.int64)
    return np.array([[tn, fp], [fn, tp]], dtype=np.int64)


def save_metrics(metrics, filename: str = "client1_metrics.csv", log=None) -> str:
    if log:
        log("Starting to save metrics")
    d = os.path.dirname(filename)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(filename, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Accuracy", "Loss", "Precision", "Recall", "F1-Score"])
        w.writerow([repr(float(metrics[0])), repr(float(metrics[1])), repr(float(metrics[2])),
                    repr(float(metrics[3])), repr(float(metrics[4]))])
    if log and hasattr(log, "info"):
        log.info(f"metrics saved to {filename}")
    return filename


def load_metrics(filename: str) -> dict:
    with open(filename) as f:
        rows = list(csv.DictReader(f))
    return {k: float(v) for k, v in rows[0].items()}
