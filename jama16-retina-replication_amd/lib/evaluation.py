"""Drop-in for the reference's lib/evaluation.py (lib/evaluation.py:1-81).

perform_test(sess, init_op, summary_writer=None, epoch=None,
             feed_dict_fn=None, feed_dict_args={}, custom_tensors=[])
keeps its arguments and outputs:
  * default path (lib/evaluation.py:20-37, 48-57, 66-81): reset the
    tp/fp/fn/tn/brier/auc streaming metrics, run every batch of `init_op`
    (the dataset to evaluate; iterating it is `sess.run(init_op)`), print
    "Brier score: {:6.4}, AUC: {:10.8}" and the confusion matrix, write the
    'auc' scalar summary at `epoch`, return the AUC;
  * custom_tensors (lib/evaluation.py:62-64): names of per-batch outputs
    ("predictions", "labels", "logits"); returns [np.vstack(...)] per name.
  * feed_dict_fn(**feed_dict_args), if given, supplies each batch as
    {"x": images, "y": labels} (evaluate.py:114-118 feed_images); raising
    StopIteration ends the pass (the OutOfRangeError of the reference).
`sess` is a jr.session.Session (engine + metric states).
"""
from __future__ import annotations

import numpy as np


def _batches(init_op, feed_dict_fn, feed_dict_args):
    if feed_dict_fn is None:
        yield from init_op
        return
    while True:
        try:
            fd = feed_dict_fn(**feed_dict_args)
        except StopIteration:
            return
        yield fd["x"], fd["y"]


def perform_test(sess, init_op, summary_writer=None, epoch=None,
                 feed_dict_fn=None, feed_dict_args={}, custom_tensors=[]):
    if len(custom_tensors) == 0:
        sess.reset("tp", "fp", "fn", "tn", "brier", "auc")

    batch_results = []
    for images, labels in _batches(init_op, feed_dict_fn, feed_dict_args):
        probs = sess.predict(images, labels)
        if len(custom_tensors) == 0:
            sess.update(labels, probs, "tp", "fp", "fn", "tn", "brier", "auc")
        else:
            out = []
            for name in custom_tensors:
                if name in ("predictions", "predictions:0", "predictions/Sigmoid:0"):
                    out.append(probs)
                elif name in ("labels", "y", "y:0"):
                    out.append(np.asarray(labels, np.float32).reshape(len(probs), -1))
                elif name == "logits":
                    out.append(sess.engine.logits[:len(probs)].cpu().numpy().reshape(len(probs), -1))
                else:
                    raise KeyError(f"unknown tensor {name!r}")
            batch_results.append(out)

    if len(custom_tensors) > 0:
        if not batch_results:
            return [np.zeros((0, 1), np.float32) for _ in custom_tensors]
        return [np.vstack(x) for x in zip(*batch_results)]

    # data-parallel ranks each ran their own batches: sum the metric states
    # (no-op for one process) so every rank reads the same Brier / AUC
    sync = getattr(sess, "sync_metrics", None)
    if sync is not None:
        sync("tp", "fp", "fn", "tn", "brier", "auc")
    test_conf_matrix = sess.confusion_matrix()
    test_brier = sess.value("brier")
    test_auc = sess.value("auc")

    if summary_writer is not None:
        summary_writer.add_summary({"auc": test_auc}, epoch)

    # data parallel: one copy of the reference's lines (rank 0; every rank
    # holds the same summed values)
    if getattr(sess, "rank", 0) == 0:
        print(f"Brier score: {test_brier:6.4}, AUC: {test_auc:10.8}")
        print(f"Confusion matrix:")
        print(test_conf_matrix[0])
    return test_auc
