"""lib/metrics.py (product host logic) against the oracle restatement and
the committed golden vectors; streaming semantics (batch-wise updates equal
one big update; reset)."""
import os

import numpy as np

from conftest import GOLDEN
from oracle import metrics_ref as MR


def test_generate_thresholds_matches_reference_formula():
    import lib.metrics as M
    assert M.generate_thresholds(200, 1e-7) == MR.generate_thresholds(200, 1e-7)
    t = M.generate_thresholds(5, 1e-3)
    assert t == [-1e-3, 0.25, 0.5, 0.75, 1 - 1e-3]


def test_streaming_metrics_equal_golden_in_batches():
    import lib.metrics as M
    m = np.load(os.path.join(GOLDEN, "metrics.npz"))
    thr = list(m["thresholds"])
    st = {k: M.create_reset_metric(f, scope=k, thresholds=thr) for k, f in (
        ("tp", M.true_positives_at_thresholds), ("fp", M.false_positives_at_thresholds),
        ("fn", M.false_negatives_at_thresholds), ("tn", M.true_negatives_at_thresholds))}
    st["brier"] = M.create_reset_metric(M.mean_squared_error, scope="brier")
    st["auc"] = M.create_reset_metric(M.auc, scope="auc")
    y, p = m["labels"], m["preds"]
    for value, update, reset in st.values():
        update(y[:10], p[:10])
        reset()                                   # reset really clears
        for s in range(0, len(y), 64):            # 64-image batches, last partial
            update(y[s:s + 64], p[s:s + 64])
    for k in ("tp", "fp", "fn", "tn"):
        np.testing.assert_array_equal(st[k][0](), m[k])
    assert abs(st["auc"][0]() - float(m["auc"])) < 2e-6
    assert abs(st["brier"][0]() - float(m["brier"])) < 1e-6
    tp, fp, fn, tn = (st[k][0]() for k in ("tp", "fp", "fn", "tn"))
    cm = M.confusion_matrix(tp[-1], fp[-1], fn[-1], tn[-1])
    assert cm.dtype == np.int32 and cm.shape == (1, 2, 2)
    np.testing.assert_array_equal(cm, m["confusion"])
    spec = tn / (tn + fp + np.float32(1e-7))
    sens = tp / (tp + fn + np.float32(1e-7))
    np.testing.assert_allclose(spec, m["spec"], rtol=1e-6)
    np.testing.assert_allclose(sens, m["sens"], rtol=1e-6)


def test_metrics_random_cases_match_oracle():
    import lib.metrics as M
    rng = np.random.default_rng(3)
    for n in (1, 7, 500):
        y = (rng.random(n) < 0.2).astype(np.float32)
        p = rng.random(n).astype(np.float32)
        v, up, _ = M.create_reset_metric(M.auc, scope="auc")
        up(y, p)
        assert abs(v() - MR.auc(y, p)) < 1e-6
        thr = MR.generate_thresholds(200) + [0.3]
        ref = MR.counts_at_thresholds(y, p, thr)
        for f, r in zip((M.true_positives_at_thresholds, M.false_positives_at_thresholds,
                         M.false_negatives_at_thresholds, M.true_negatives_at_thresholds), ref):
            v, up, _ = M.create_reset_metric(f, thresholds=thr)
            up(y, p)
            np.testing.assert_array_equal(v(), r)
