"""train.py as the drop-in for data-parallel training (BASELINE configs 2/3:
`torchrun --nproc-per-node N train.py ...`, the reference's multi-GPU run is
`--num_gpus=N --batch_size=64`, /root/reference/README.md:76).

Two ranks of the real CLI (gloo, both on cuda:0 -- RCCL refuses two ranks on
one device, the one-GPU box has one) train 2 epochs at 107^2 in f32 (x8) and
bf16.  Checked:
  * the two ranks' parameters after every epoch are byte-identical (and
    train.py's own per-epoch digest check passed);
  * the parameters after epoch 0 equal ONE process that steps the same two
    shards of the same seeded stream (batch 2s on rank 0, 2s+1 on rank 1),
    sums their gradients (fp32 a + b, the two-rank all-reduce) and applies
    Nesterov with grad_scale 1/2 -- the test_gpu_dp.py construction;
  * only rank 0 prints the reference's status / early-stop lines, and its
    op-point CSV has the header + 200 rows (train.py:287-300).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu

RES, NTRAIN, NVAL, B = 107, 256, 64, 64


@pytest.fixture(scope="module")
def records(tmp_path_factory):
    from jr import synth_records
    d = tmp_path_factory.mktemp("dp_train")
    synth_records.write_split(str(d / "train"), NTRAIN, size=RES, num_shards=2, name="train")
    synth_records.write_split(str(d / "val"), NVAL, size=RES, start=1000, num_shards=1, name="validation")
    return d


def _one_process_epoch0(train_dir, dtype, seed, shuffle_seed):
    """Epoch 0 of the two-rank job in one process."""
    import torch
    import lib.dataset
    from jr.engine import Engine
    eng = Engine(B, RES, RES, device=0, optimizer="nesterov", lr=3e-3, momentum=0.9, seed=seed, dtype=dtype,
                 conv_math="x6h" if dtype == "f32" else "bf16", tiles="pinned")   # train.py's defaults
    ds = lib.dataset.initialize_dataset(train_dir, B, num_workers=8, prefetch_buffer_size=2 * B,
                                        shuffle_buffer_size=2048, image_data_format="channels_last",
                                        num_channels=3, image_dim=[RES, RES], seed=shuffle_seed,
                                        decode_dtype="uint8")
    it = iter(ds)
    batches = [b for b in it]
    lib.dataset.close_iterator(it)
    assert len(batches) == NTRAIN // B
    steps = -(-NTRAIN // B) // 2            # train.py: steps per epoch per rank
    for s in range(steps):
        gsum = None
        for r in range(2):
            x, y = batches[2 * s + r]
            eng.set_batch(x, y)
            eng.forward()
            eng.backward()
            eng.synchronize()
            g = eng.grads.clone()
            gsum = g if gsum is None else gsum + g
        eng.grads.copy_(gsum)
        torch.cuda.synchronize()
        eng.apply_update(grad_scale=0.5)
    return eng.params_numpy()


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_train_cli_two_ranks(records, tmp_path, dtype):
    d = records
    out = tmp_path / "out"
    dump = tmp_path / "replicas"
    logs = tmp_path / "torchrun_logs"
    port = 29600 + (os.getpid() + (7 if dtype == "bf16" else 0)) % 1000
    seed, shuffle_seed = 2, 5
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([PKG, ROOT]), JR_DIST_BACKEND="gloo", JR_ONE_DEVICE="1")
    args = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
            "--master-addr", "127.0.0.1", "--master-port", str(port), "--log-dir", str(logs), "--redirects", "3",
            os.path.join(PKG, "train.py"), "-t", str(d / "train"), "-v", str(d / "val"),
            "-sm", str(out / "model"), "-ss", str(out / "logs"), "-so", str(out / "op.csv"),
            "--image_size", str(RES), "--num_epochs", "2", "--seed", str(seed), "--shuffle_seed", str(shuffle_seed),
            "--dtype", dtype, "--replica_dump_dir", str(dump)]
    r = subprocess.run(args, capture_output=True, text=True, env=env, cwd=str(tmp_path), timeout=900)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])

    stdout = {}
    for k in range(2):
        f = list(logs.glob(f"*/attempt_*/{k}/stdout.log"))
        assert len(f) == 1, f
        stdout[k] = f[0].read_text()
    assert "End of epoch 0!" in stdout[0] and "End of epoch 1!" in stdout[0]
    assert "Brier score:" in stdout[0] and "AUC:" in stdout[0]
    assert "New peak auc reached" in stdout[0] or "Stopped early" in stdout[0]
    for line in ("End of epoch", "New peak auc", "Stopped early", "Brier score:", "Confusion matrix", "Numpy version",
                 "Training images folder"):
        assert line not in stdout[1], (line, stdout[1])
    rows = open(out / "op.csv").read().strip().split("\n")
    assert rows[0] == "threshold specificity sensitivity" and len(rows) == 201

    for e in range(2):
        p0 = np.load(dump / f"params_e{e}_r0.npy")
        p1 = np.load(dump / f"params_e{e}_r1.npy")
        assert p0.tobytes() == p1.tobytes(), e

    want = _one_process_epoch0(str(d / "train"), dtype, seed, shuffle_seed)
    got = np.load(dump / "params_e0_r0.npy")
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (bad.size, bad[:5], got[bad[:5]], want[bad[:5]])
