"""Evaluation plots (reference ``plot_evaluation``, client1.py:153-225), matplotlib only.

Writes the reference's three files into ``output_dir``:
``local_confusion_matrix.png``, ``aggregated_confusion_matrix.png`` (when an
aggregated result exists) and ``metrics_comparison.png`` (grouped bars of
Accuracy/Precision/Recall/F1).  seaborn is not installed here, so the heatmap is
an annotated ``imshow``.  The reference defines ROC / precision-recall plots but
never calls them (client1.py:167-193); they are available via ``curves=True``.
Titles follow the code (the committed PNGs have local/aggregated swapped).

Artefact parity, stated plainly: the figure sizes, colours (``darkorange``/``navy``/
``purple``; ``#1f77b4``/``#ff7f0e``), labels and axis limits below deliberately follow
client1.py:157-218 call for call, because the three PNGs are part of the reference's
observable output.  These are leaf matplotlib calls with no design freedom worth taking;
everything upstream of them (metrics on device, one sync) is this framework's own.
DPI: client 1 uses matplotlib's default, client 2 saves at ``dpi=300``
(client2.py:155,171,183,207) -- ``reference_dpi(client_id)``.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np


def _plt():
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    return plt


def plot_confusion_matrix(cm, title: str, path: str, dpi: Optional[int] = None):
    plt = _plt()
    cm = np.asarray(cm)
    fig, ax = plt.subplots(figsize=(6, 6))
    ax.imshow(cm, cmap="Blues")
    for i in range(cm.shape[0]):
        for j in range(cm.shape[1]):
            ax.text(j, i, f"{int(cm[i, j])}", ha="center", va="center",
                    color="white" if cm[i, j] > cm.max() / 2 else "black")
    ax.set_xticks(range(cm.shape[1]))
    ax.set_yticks(range(cm.shape[0]))
    ax.set_title(title)
    ax.set_ylabel("True Label")
    ax.set_xlabel("Predicted Label")
    fig.savefig(path, dpi=dpi)
    plt.close(fig)
    return path


def plot_roc_curve(labels, probs, title: str, path: str, dpi=None):
    from sklearn.metrics import auc, roc_curve
    plt = _plt()
    fpr, tpr, _ = roc_curve(labels, probs)
    fig = plt.figure(figsize=(8, 6))
    plt.plot(fpr, tpr, color="darkorange", lw=2, label=f"ROC curve (AUC = {auc(fpr, tpr):.2f})")
    plt.plot([0, 1], [0, 1], color="navy", lw=2, linestyle="--")
    plt.xlim([0.0, 1.0])
    plt.ylim([0.0, 1.05])
    plt.xlabel("False Positive Rate")
    plt.ylabel("True Positive Rate")
    plt.title(title)
    plt.legend(loc="lower right")
    fig.savefig(path, dpi=dpi)
    plt.close(fig)
    return path


def plot_precision_recall_curve(labels, probs, title: str, path: str, dpi=None):
    from sklearn.metrics import precision_recall_curve
    plt = _plt()
    precision, recall, _ = precision_recall_curve(labels, probs)
    fig = plt.figure(figsize=(8, 6))
    plt.plot(recall, precision, color="purple", lw=2, label="Precision-Recall curve")
    plt.xlabel("Recall")
    plt.ylabel("Precision")
    plt.title(title)
    plt.legend(loc="lower left")
    fig.savefig(path, dpi=dpi)
    plt.close(fig)
    return path


def plot_metrics_comparison(local_metrics, aggregated_metrics, path: str, client_name: str = "Client 1", dpi=None):
    plt = _plt()
    names = ["Accuracy", "Precision", "Recall", "F1-Score"]
    lv = [local_metrics[0], local_metrics[2], local_metrics[3], local_metrics[4]]
    x = np.arange(len(names))
    fig, ax = plt.subplots(figsize=(10, 6))
    if aggregated_metrics is not None:
        av = [aggregated_metrics[0], aggregated_metrics[2], aggregated_metrics[3], aggregated_metrics[4]]
        w = 0.35
        ax.bar(x - w / 2, lv, w, label="Local Model", color="#1f77b4")
        ax.bar(x + w / 2, av, w, label="Aggregated Model", color="#ff7f0e")
        ax.set_title(f"{client_name}: Local vs Aggregated Model Performance")
    else:
        ax.bar(x, lv, label="Local Model", color="#1f77b4")
        ax.set_title(f"{client_name}: Local Model Performance")
    ax.set_ylabel("Value")
    ax.set_xticks(x)
    ax.set_xticklabels(names)
    ax.legend()
    fig.savefig(path, dpi=dpi)
    plt.close(fig)
    return path


def reference_dpi(client_id: int) -> Optional[int]:
    """The reference's per-client DPI: client1.py saves at the default, client2.py at 300."""
    return None if int(client_id) == 1 else 300


def plot_evaluation(local_metrics, aggregated_metrics=None, output_dir: str = "client1_plots",
                    client_name: str = "Client 1", curves: bool = False, dpi: Optional[int] = None, log=None):
    if log:
        log.phase("Starting plot generation")
    os.makedirs(output_dir, exist_ok=True)
    out = [plot_confusion_matrix(local_metrics[5], f"{client_name} Local Model Confusion Matrix",
                                 os.path.join(output_dir, "local_confusion_matrix.png"), dpi)]
    if aggregated_metrics is not None:
        out.append(plot_confusion_matrix(aggregated_metrics[5], f"{client_name} Aggregated Model Confusion Matrix",
                                         os.path.join(output_dir, "aggregated_confusion_matrix.png"), dpi))
    out.append(plot_metrics_comparison(local_metrics, aggregated_metrics,
                                       os.path.join(output_dir, "metrics_comparison.png"), client_name, dpi))
    if curves:
        m = aggregated_metrics if aggregated_metrics is not None else local_metrics
        if len(set(m[6])) == 2:
            out.append(plot_roc_curve(m[6], m[7], f"{client_name} ROC", os.path.join(output_dir, "roc_curve.png"), dpi))
            out.append(plot_precision_recall_curve(m[6], m[7], f"{client_name} Precision-Recall",
                                                   os.path.join(output_dir, "precision_recall_curve.png"), dpi))
    if log:
        for p in out:
            log.info(f"{os.path.basename(p)} saved to {output_dir}")
        log.phase("Finished plot generation")
    return out


def plot_scaling(results, path: str, dpi=None):
    """Scaling curve: batches/s per client and aggregate vs number of GPUs."""
    plt = _plt()
    ns = [r["n_gpus"] for r in results]
    per = [r["per_client_batches_per_sec"] for r in results]
    agg = [r["value"] for r in results]
    fig, ax = plt.subplots(figsize=(8, 5))
    ax.plot(ns, agg, "o-", label="aggregate batches/s")
    ax.plot(ns, per, "s--", label="per-client batches/s")
    ax.set_xlabel("GPUs (clients)")
    ax.set_ylabel("batches/s (bs32, seq128)")
    ax.set_xticks(ns)
    ax.legend()
    ax.grid(alpha=0.3)
    fig.savefig(path, dpi=dpi)
    plt.close(fig)
    return path
