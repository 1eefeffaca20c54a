"""Restatement of the reference's TF streaming metrics (TEST ORACLE ONLY).

Parity unpinned (oracle/__init__.py).  Follows:
  lib/metrics.py:4-8    generate_thresholds
  lib/metrics.py:20-24  confusion_matrix -> int32 [1,2,2] of [[tp,fp],[fn,tn]]
  train.py:156-184 / evaluate.py:128-161  tf.metrics.{true,false}_{positives,
      negatives}_at_thresholds, mean_squared_error, auc, and the
      specificity / sensitivity tf.div expressions
  [TF-3P] metrics_impl._confusion_matrix_at_thresholds (pred > thr, strict;
      float32 accumulators) and metrics_impl.auc (num_thresholds=200, ROC,
      trapezoidal, eps 1e-6, own thresholds ending at 1 + 1e-7).
Deliberately loop-based (one threshold at a time) so it shares no code shape
with the vectorised product implementation in lib/metrics.py.
"""
from __future__ import annotations

import numpy as np


def generate_thresholds(num_thresholds: int, kepsilon: float = 1e-7):
    inner = [(i + 1) * 1.0 / (num_thresholds - 1) for i in range(num_thresholds - 2)]
    return [0.0 - kepsilon] + inner + [1.0 - kepsilon]


def counts_at_thresholds(labels, predictions, thresholds):
    """tp, fp, fn, tn (float32) per threshold; positive iff pred > thr."""
    y = np.asarray(labels).reshape(-1).astype(bool)
    p = np.asarray(predictions, np.float32).reshape(-1)
    out = np.zeros((4, len(thresholds)), np.float32)
    for i, t in enumerate(thresholds):
        pos = p > np.float32(t)
        out[0, i] = np.sum(pos & y)
        out[1, i] = np.sum(pos & ~y)
        out[2, i] = np.sum(~pos & y)
        out[3, i] = np.sum(~pos & ~y)
    return out[0], out[1], out[2], out[3]


def auc(labels, predictions, num_thresholds: int = 200):
    """tf.metrics.auc default (ROC, trapezoidal), in float32 like TF."""
    kepsilon = 1e-7
    thr = [(i + 1) * 1.0 / (num_thresholds - 1) for i in range(num_thresholds - 2)]
    thr = [0.0 - kepsilon] + thr + [1.0 + kepsilon]
    tp, fp, fn, tn = counts_at_thresholds(labels, predictions, thr)
    eps = np.float32(1e-6)
    rec = (tp + eps) / (tp + fn + eps)
    fpr = fp / (fp + tn + eps)
    total = np.float32(0.0)
    for i in range(num_thresholds - 1):
        total += (fpr[i] - fpr[i + 1]) * (rec[i] + rec[i + 1]) / np.float32(2.0)
    return float(total)


def brier(labels, predictions):
    """tf.metrics.mean_squared_error (train.py:175-177)."""
    y = np.asarray(labels, np.float64).reshape(-1)
    p = np.asarray(predictions, np.float64).reshape(-1)
    return float(np.mean((p - y) ** 2))


def spec_sens(tp, fp, fn, tn, kepsilon: float = 1e-7):
    """train.py:183-184: tn/(tn+fp+eps), tp/(tp+fn+eps)."""
    k = np.float32(kepsilon)
    return tn / (tn + fp + k), tp / (tp + fn + k)


def confusion_matrix(tp, fp, fn, tn):
    """lib/metrics.py:20-24 at the operating threshold (index -1)."""
    return np.array([tp, fp, fn, tn], np.float32).reshape(1, 2, 2).astype(np.int32)
