"""Checkpoint format, ensemble path expansion, and the CLI surface of the
drop-in train.py / evaluate.py (flags of train.py:29-46, evaluate.py:31-49)."""
import os

import numpy as np
import pytest


def test_checkpoint_roundtrip_and_glob_semantics(tmp_path):
    from jr import checkpoint
    from jr.inception import build_inception_v3
    from jr.init import init_params
    g = build_inception_v3(107, 107)
    flat = init_params(g, 2)
    for m in range(3):
        checkpoint.save(str(tmp_path / f"model_{m}"), g, flat + m, {"epoch": m})
    got, meta = checkpoint.load(str(tmp_path / "model_1"), g)
    np.testing.assert_array_equal(got, flat + 1)
    assert meta["height"] == 107 and meta["epoch"] == 1
    import evaluate
    paths = evaluate.expand_model_paths(str(tmp_path / "model_?"))
    assert paths == [str(tmp_path / f"model_{m}") for m in range(3)]
    assert evaluate.expand_model_paths("a,b") == ["a", "b"]
    assert evaluate.expand_model_paths("plain") == ["plain"]
    # corrupted data is refused
    p = str(tmp_path / "model_2") + checkpoint.DATA_SUFFIX
    raw = bytearray(open(p, "rb").read())
    raw[100] ^= 0xFF
    open(p, "wb").write(bytes(raw))
    with pytest.raises(ValueError):
        checkpoint.load(str(tmp_path / "model_2"))
    with pytest.raises(ValueError):
        checkpoint.load(str(tmp_path / "model_0"), build_inception_v3(107, 107, units=2))


def test_train_cli_flags_and_defaults():
    import train
    a = train.build_parser().parse_args([])
    assert (a.train_dir, a.val_dir, a.save_model_path, a.save_summaries_dir, a.save_operating_thresholds_path,
            a.vanilla_sgd) == ("./data/eyepacs/bin2/train", "./data/eyepacs/bin2/validation", "./tmp/model",
                               "./tmp/logs", "./tmp/op_pts.csv", False)
    a = train.build_parser().parse_args(["-t", "T", "-v", "V", "-sm", "M", "-ss", "S", "-so", "O", "-sgd"])
    assert (a.train_dir, a.val_dir, a.save_model_path, a.save_summaries_dir, a.save_operating_thresholds_path,
            a.vanilla_sgd) == ("T", "V", "M", "S", "O", True)
    assert (train.LEARNING_RATE, train.MOMENTUM, train.TRAIN_BATCH_SIZE, train.NUM_EPOCHS, train.WAIT_EPOCHS,
            train.MIN_DELTA_AUC, train.SHUFFLE_BUFFER_SIZE) == (3e-3, 0.9, 64, 200, 10, 0.01, 2048)
    s = train.status_line(3, 200, 7, 0.693147, 1234)
    assert s == "Epoch:   3/200, Batch:    7, Xent: 0.6931, Step:       1234"


def test_evaluate_cli_flags_and_dataset_selection(capsys):
    import evaluate
    a = evaluate.build_parser().parse_args(["-e", "-lm", "x,y", "-b", "16", "-op", "0.3"])
    assert a.eyepacs and a.load_model_path == "x,y" and int(a.batch_size) == 16
    assert float(a.operating_threshold) == 0.3
    d = evaluate.build_parser().parse_args([])
    assert (d.load_model_path, d.save_operating_thresholds_path, d.batch_size, d.operating_threshold) == (
        "./tmp/model", "./tmp/test_op_pts.csv", 32, 0.5)
    # none or all three dataset flags: refused (evaluate.py:53-56)
    assert evaluate.main([]) == 2
    assert evaluate.main(["-e", "-m", "-o"]) == 2
    assert evaluate.main(["-o"]) == 2            # -o without --data_dir
    assert "Please specify --data_dir." in capsys.readouterr().out


def test_summary_writer_writes_tfrecord_events(tmp_path):
    from jr import summary, tfrecord
    w = summary.FileWriter(str(tmp_path))
    w.add_summary({"auc": 0.75}, 3)
    w.close()
    recs = list(tfrecord.read_records(w.path))
    assert len(recs) == 2 and b"brain.Event:2" in recs[0] and b"auc" in recs[1]


def test_glob_ignores_incomplete_checkpoints(tmp_path):
    """A leftover `.data-*.tmp` of an interrupted save strips to
    `<path>.data-00000-of-00001`, which is not a checkpoint: dropped."""
    import evaluate
    from jr import checkpoint
    from jr.inception import build_inception_v3
    from jr.init import init_params
    g = build_inception_v3(75, 75)
    checkpoint.save(str(tmp_path / "model_1"), g, init_params(g, 1))
    open(str(tmp_path / "model_2") + checkpoint.DATA_SUFFIX + ".tmp", "wb").write(b"partial")
    assert evaluate.expand_model_paths(str(tmp_path / "model_*")) == [str(tmp_path / "model_1")]
    meta = checkpoint.read_meta(str(tmp_path / "model_1"))
    assert (meta["height"], meta["width"]) == (75, 75)
