"""Drop-in for the reference's lib/metrics.py (lib/metrics.py:1-24), no TF.

generate_thresholds and confusion_matrix keep their signatures and results.
create_reset_metric keeps its signature `(metric, scope, **metric_args)` and
its (value, update, reset) triple; without a TF graph the three are
callables on a host-side streaming state:
    value()                      -> current metric value
    update(labels, predictions)  -> accumulate one batch, returns the value
    reset()                      -> tf.variables_initializer(local vars)
`metric` is one of the tf.metrics restatements below (same names and
keyword arguments as the TF functions the reference passes: train.py:156-180,
evaluate.py:128-161): labels/predictions given at construction are ignored
(they were graph tensors); the batch arrays are passed to update().

Arithmetic follows [TF-3P] metrics_impl: `_confusion_matrix_at_thresholds`
(labels -> bool, positive iff prediction > threshold, float32 counters),
`auc` (num_thresholds=200, ROC, trapezoidal, its own thresholds
[-1e-7, (i+1)/199 ..., 1+1e-7], epsilon 1e-6) and `mean_squared_error`
(float32 total / count).
"""
from __future__ import annotations

from typing import Callable, Sequence, Tuple

import numpy as np


def generate_thresholds(num_thresholds, kepsilon=1e-7):
    """lib/metrics.py:4-8."""
    thresholds = [(i + 1) * 1.0 / (num_thresholds - 1) for i in range(num_thresholds - 2)]
    return [0.0 - kepsilon] + thresholds + [1.0 - kepsilon]


def _counts(labels, predictions, thresholds) -> np.ndarray:
    """[4, T] float32 (tp, fp, fn, tn) of one batch; pred > thr is positive."""
    y = np.asarray(labels).reshape(-1).astype(bool)
    p = np.asarray(predictions, dtype=np.float32).reshape(-1)
    thr = np.asarray(thresholds, dtype=np.float32)
    pos = p[None, :] > thr[:, None]                      # [T, N]
    tp = np.sum(pos & y[None, :], axis=1)
    fp = np.sum(pos & ~y[None, :], axis=1)
    fn = np.sum(~pos & y[None, :], axis=1)
    tn = np.sum(~pos & ~y[None, :], axis=1)
    return np.stack([tp, fp, fn, tn]).astype(np.float32)


class _StreamingMetric:
    """Local-variable state of one tf.metrics op."""

    def reset(self) -> None:
        raise NotImplementedError

    def update(self, labels, predictions):
        raise NotImplementedError

    def value(self):
        raise NotImplementedError


class _AtThresholds(_StreamingMetric):
    ROW = 0

    def __init__(self, labels=None, predictions=None, thresholds: Sequence[float] = (0.5,), **_):
        self.thresholds = list(thresholds)
        self.reset()

    def reset(self):
        self.acc = np.zeros(len(self.thresholds), np.float32)

    def update(self, labels, predictions):
        self.acc = self.acc + _counts(labels, predictions, self.thresholds)[self.ROW]
        return self.acc.copy()

    def value(self):
        return self.acc.copy()


class true_positives_at_thresholds(_AtThresholds):
    ROW = 0


class false_positives_at_thresholds(_AtThresholds):
    ROW = 1


class false_negatives_at_thresholds(_AtThresholds):
    ROW = 2


class true_negatives_at_thresholds(_AtThresholds):
    ROW = 3


class mean_squared_error(_StreamingMetric):
    """tf.metrics.mean_squared_error: total / count (float32 locals)."""

    def __init__(self, labels=None, predictions=None, **_):
        self.reset()

    def reset(self):
        self.total = np.float32(0.0)
        self.count = np.float32(0.0)

    def update(self, labels, predictions):
        y = np.asarray(labels, np.float32).reshape(-1)
        p = np.asarray(predictions, np.float32).reshape(-1)
        self.total = np.float32(self.total + np.sum((p - y) ** 2, dtype=np.float32))
        self.count = np.float32(self.count + np.float32(y.size))
        return self.value()

    def value(self):
        return float(self.total / self.count) if self.count > 0 else 0.0


class auc(_StreamingMetric):
    """tf.metrics.auc(num_thresholds=200, curve='ROC', trapezoidal)."""

    def __init__(self, labels=None, predictions=None, num_thresholds: int = 200, curve: str = "ROC", **_):
        if curve != "ROC":
            raise NotImplementedError("only curve='ROC' is used by the reference")
        self.num_thresholds = num_thresholds
        kepsilon = 1e-7
        inner = [(i + 1) * 1.0 / (num_thresholds - 1) for i in range(num_thresholds - 2)]
        self.thresholds = [0.0 - kepsilon] + inner + [1.0 + kepsilon]
        self.reset()

    def reset(self):
        self.acc = np.zeros((4, self.num_thresholds), np.float32)

    def update(self, labels, predictions):
        p = np.asarray(predictions, np.float32)
        if p.size and (p.min() < 0 or p.max() > 1):
            raise ValueError("auc: predictions must be in [0, 1]")
        self.acc = self.acc + _counts(labels, p, self.thresholds)
        return self.value()

    def value(self):
        tp, fp, fn, tn = self.acc
        eps = np.float32(1e-6)
        rec = (tp + eps) / (tp + fn + eps)
        fpr = fp / (fp + tn + eps)
        n = self.num_thresholds
        return float(np.sum((fpr[:n - 1] - fpr[1:]) * (rec[:n - 1] + rec[1:]) / np.float32(2.0),
                            dtype=np.float32))


def create_reset_metric(metric, scope='reset_metrics', **metric_args) -> Tuple[Callable, Callable, Callable]:
    """lib/metrics.py:11-17: (metric value, update op, reset op)."""
    state = metric(**metric_args)
    state.scope = scope
    return state.value, state.update, state.reset


def confusion_matrix(tp, fp, fn, tn, num_labels=1, scope='confusion_matrix'):
    """lib/metrics.py:20-24: int32 [num_labels, 2, 2] of [[tp, fp], [fn, tn]]."""
    return np.reshape(np.stack([np.asarray(tp, np.float32), np.asarray(fp, np.float32),
                                np.asarray(fn, np.float32), np.asarray(tn, np.float32)], 0),
                      [num_labels, 2, 2]).astype(np.int32)
