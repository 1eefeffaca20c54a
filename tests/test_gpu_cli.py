"""End-to-end drop-in run on the GPU: synthetic TFRecords -> train.py (2
epochs, early-stopping bookkeeping, checkpoint, op-point CSV) -> evaluate.py
with a 2-model glob ensemble (-lm), at 107^2 to stay small."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import PKG

pytestmark = pytest.mark.gpu


def _run(args, cwd):
    r = subprocess.run([sys.executable] + args, cwd=cwd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def test_train_then_ensemble_evaluate(tmp_path):
    from jr import synth_records
    d = tmp_path / "data"
    synth_records.write_split(str(d / "train"), 24, size=107, num_shards=2, name="train")
    synth_records.write_split(str(d / "val"), 12, size=107, start=100, num_shards=1, name="validation")
    synth_records.write_split(str(d / "test"), 20, size=107, start=200, num_shards=2, name="test",
                              p=0.3, label_seed=11)
    out = tmp_path / "out"
    for m in range(2):
        log = _run([os.path.join(PKG, "train.py"), "-t", str(d / "train"), "-v", str(d / "val"),
                    "-sm", str(out / f"model_{m}"), "-ss", str(out / "logs"), "-so", str(out / f"op_{m}.csv"),
                    "--image_size", "107", "--num_epochs", "2", "--seed", str(m), "--shuffle_seed", "1"],
                   cwd=str(tmp_path))
        assert "End of epoch 0!" in log and "Brier score:" in log and "AUC:" in log
        rows = open(out / f"op_{m}.csv").read().strip().split("\n")
        assert rows[0] == "threshold specificity sensitivity" and len(rows) == 201
    log = _run([os.path.join(PKG, "evaluate.py"), "-o", "--data_dir", str(d / "test"),
                "-lm", str(out / "model_*"), "-b", "8", "-so", str(out / "test_op.csv")], cwd=str(tmp_path))
    assert "Trying to load model(s):" in log and "model_0" in log and "model_1" in log
    assert "Confusion matrix at operating threshold 0.500" in log
    assert "Specificity:" in log and "Sensitivity:" in log
    rows = open(out / "test_op.csv").read().strip().split("\n")
    assert len(rows) == 201
    vals = np.array([[float(v) for v in r.split()] for r in rows[1:]])
    assert np.all((vals[:, 1:] >= 0) & (vals[:, 1:] <= 1))
