"""Evaluation plots (reference: core/src/main/python/synapse/ml/plot/plot.py:
``confusionMatrix(df, y_col, y_hat_col, labels)``, ``roc(df, y_col,
y_hat_col, thresh)``). Returns the matplotlib figure (Agg backend, no
display needed) and the underlying numbers."""
from __future__ import annotations

from typing import Sequence

import numpy as np


def _plt():
    import matplotlib

    matplotlib.use("Agg", force=False)
    import matplotlib.pyplot as plt

    return plt


def confusionMatrix(df, y_col: str, y_hat_col: str, labels: Sequence):  # noqa: N802
    y = np.asarray(df[y_col], dtype=np.float64).astype(int)
    yh = np.asarray(df[y_hat_col], dtype=np.float64).astype(int)
    k = len(labels)
    cm = np.zeros((k, k), dtype=np.int64)
    for a, b in zip(y, yh):
        if 0 <= a < k and 0 <= b < k:
            cm[a, b] += 1
    norm = cm / np.maximum(cm.sum(1, keepdims=True), 1)
    plt = _plt()
    fig, ax = plt.subplots(figsize=(4, 4))
    ax.imshow(norm, cmap="Blues", vmin=0, vmax=1)
    ax.set_xticks(range(k), labels=list(labels))
    ax.set_yticks(range(k), labels=list(labels))
    for i in range(k):
        for j in range(k):
            ax.text(j, i, f"{norm[i, j]:.2f}", ha="center", va="center")
    ax.set_xlabel("Predicted")
    ax.set_ylabel("Actual")
    acc = np.trace(cm) / max(1, cm.sum())
    ax.set_title(f"Accuracy: {acc:.3f}")
    return fig, cm


def roc(df, y_col: str, y_hat_col: str, thresh: float = 0.5):
    from ..models.evaluation import auc, roc_curve

    y = (np.asarray(df[y_col], dtype=np.float64) > thresh).astype(np.float64)
    s = np.asarray(df[y_hat_col], dtype=np.float64)
    if s.ndim == 2:
        s = s[:, -1]
    fpr, tpr = roc_curve(y, s)
    a = auc(y, s)
    plt = _plt()
    fig, ax = plt.subplots(figsize=(4, 4))
    ax.plot(fpr, tpr, label=f"AUC = {a:.3f}")
    ax.plot([0, 1], [0, 1], "k--", linewidth=0.8)
    ax.set_xlabel("False positive rate")
    ax.set_ylabel("True positive rate")
    ax.legend(loc="lower right")
    return fig, (fpr, tpr, a)


__all__ = ["confusionMatrix", "roc"]
