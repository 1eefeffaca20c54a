"""Session: what the reference's tf.Session + graph bundle held.

train.py:99-184 builds, in one graph: the model replica (x:0 -> predictions:0),
the loss, the optimizer step, and streaming metrics named tp/fp/fn/tn/brier/
auc over `thresholds` (looked up by name in lib/evaluation.py:20-37).  Here
the replica is a jr.Engine on one GPU and the metrics are lib.metrics
states; `run_*` methods are the sess.run calls of the reference.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from lib import metrics as M


class Session:
    def __init__(self, engine, thresholds=None, num_thresholds: int = 200, kepsilon: float = 1e-7):
        self.engine = engine
        if thresholds is None:
            thresholds = M.generate_thresholds(num_thresholds, kepsilon) + [0.5]
        self.thresholds = list(thresholds)
        self.num_thresholds = num_thresholds
        self.kepsilon = kepsilon
        self.metrics = {
            "tp": M.create_reset_metric(M.true_positives_at_thresholds, scope="tp", thresholds=self.thresholds),
            "fp": M.create_reset_metric(M.false_positives_at_thresholds, scope="fp", thresholds=self.thresholds),
            "fn": M.create_reset_metric(M.false_negatives_at_thresholds, scope="fn", thresholds=self.thresholds),
            "tn": M.create_reset_metric(M.true_negatives_at_thresholds, scope="tn", thresholds=self.thresholds),
            "brier": M.create_reset_metric(M.mean_squared_error, scope="brier"),
            "auc": M.create_reset_metric(M.auc, scope="auc"),
        }
        self.global_step = 0
        # data-parallel ranks: reduce(vec float64) -> elementwise sum over ranks;
        # rank: only rank 0 prints the reference's per-pass lines
        self.reduce = None
        self.rank = 0

    def sync_metrics(self, *names) -> None:
        """Sum the streaming states of `names` over the ranks (collective: every
        rank calls it at the same point).  The states are counts and sums
        (tp/fp/fn/tn at thresholds, the AUC's own confusion counts, Brier
        total and count), so the reduced state is the state of one pass over
        every rank's batches, and every rank then reads the same value."""
        if self.reduce is None:
            return
        objs = [self.metrics[n][0].__self__ for n in names]
        parts = []
        for o in objs:
            parts += [np.ravel(o.acc)] if hasattr(o, "acc") else [np.array([o.total, o.count])]
        vec = self.reduce(np.concatenate(parts).astype(np.float64))
        k = 0
        for o in objs:
            if hasattr(o, "acc"):
                n = o.acc.size
                o.acc = vec[k:k + n].reshape(o.acc.shape).astype(np.float32)
            else:
                n = 2
                o.total, o.count = np.float32(vec[k]), np.float32(vec[k + 1])
            k += n

    # ------------------------------------------------------------ metrics
    def reset(self, *names):
        for n in names or self.metrics:
            self.metrics[n][2]()

    def update(self, labels, probs, *names):
        for n in names or self.metrics:
            self.metrics[n][1](labels, probs)

    def value(self, name):
        return self.metrics[name][0]()

    def confusion_matrix(self):
        tp, fp, fn, tn = (self.value(k) for k in ("tp", "fp", "fn", "tn"))
        return M.confusion_matrix(tp[-1], fp[-1], fn[-1], tn[-1])

    def specificities(self):
        tn, fp = self.value("tn"), self.value("fp")
        return tn / (tn + fp + np.float32(self.kepsilon))

    def sensitivities(self):
        tp, fn = self.value("tp"), self.value("fn")
        return tp / (tp + fn + np.float32(self.kepsilon))

    # ------------------------------------------------------------- model
    def predict(self, images, labels=None) -> np.ndarray:
        """Forward of one batch with batch-statistics BN (App. C Q1):
        `predictions:0` of evaluate.py:181-184."""
        B = self.engine.set_batch(images, labels if labels is not None else np.zeros((len(images), self.engine.units), np.float32))
        self.engine.forward(B)
        return self.engine.predictions(B)

    def train_batch(self, images, labels) -> tuple:
        """train.py:231-232: one step; returns (global_step, xent, probs)."""
        B = self.engine.set_batch(images, labels)
        step = self.global_step
        self.engine.train_step(B, allreduce=getattr(self, "allreduce", None))
        self.global_step += 1
        return step, self.engine.loss_value(), self.engine.predictions(B)
