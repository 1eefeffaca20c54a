"""BASELINE config 4 at its workload geometry: the
ensemble inference of evaluate.py -lm (/root/reference/evaluate.py:166-236,
lib/evaluation.py:48-64) at 299^2 with eval batches of 32, through the
drop-in's own path: synthetic TFRecords -> lib.dataset (native JPEG decode)
-> evaluate.make_engines (one engine per member, the PINNED eval tile table)
-> evaluate.predict_all -> linear mean -> TF metrics.

Against the committed fp64 fixture tests/golden/eval_res299_b32.npz
(oracle/make_golden.py eval299: 3 members x 280 images, the last batch 24,
batch-statistics BN per batch, App. C Q1):
  * the decoded inputs are the fixture's (sha256 over every pixel);
  * fp32 (x8): every prediction within 1e-4 of fp64 and the ensemble AUC
    equal to 3 decimals (north_star), Brier within 1e-5, the confusion
    matrix at the 0.5 operating point equal;
  * bf16 (configs 3/5's arithmetic, not the reference's eval precision):
    bounded by the emulated-bf16 oracle's gap to fp64 on the same fixture
    (an independent bf16 implementation): max prediction error <= 3x its
    gap, AUC and Brier gaps <= 3x its gaps (+ small floors);
  * the CLI on two ranks (gloo, one device: JR_DIST_BACKEND / JR_ONE_DEVICE)
    prints the same lines and writes the same CSV, byte for byte, as on one
    rank (evaluate.py's rank-sharded batches + gather, evaluate.py:195-211
    of the drop-in)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, PKG, ROOT

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

G = np.load(os.path.join(GOLDEN, "eval_res299_b32.npz"))
B = int(G["batch"])


@pytest.fixture(scope="module")
def evalset(tmp_path_factory):
    from jr import checkpoint
    from jr.inception import build_inception_v3
    from jr.init import init_params
    from oracle import make_golden
    d = tmp_path_factory.mktemp("eval299")
    data = str(d / "test")
    make_golden.eval_records(data)
    g = build_inception_v3(int(G["res"]), int(G["res"]))
    paths = []
    for m in range(int(G["members"])):
        p = str(d / f"model_{m}")
        checkpoint.save(p, g, init_params(g, m))
        paths.append(p)
    return data, paths, d


def _metrics(labels, ens):
    from oracle import metrics_ref as MR
    thr = MR.generate_thresholds(200, 1e-7) + [0.5]
    tp, fp, fn, tn = MR.counts_at_thresholds(labels, ens, thr)
    return MR.auc(labels, ens), MR.brier(labels, ens), MR.confusion_matrix(tp[-1], fp[-1], fn[-1], tn[-1])


def test_inputs_match_the_fixture(evalset):
    from oracle import make_golden
    data, _, _ = evalset
    _, ys, digest = make_golden.eval_batches(data, B)
    assert digest == str(G["input_sha256"]), "decoded test images differ from the fixture's"
    assert np.array_equal(np.vstack(ys), G["labels"])


@pytest.mark.parametrize("grouped", [True, False], ids=["grouped", "per_member"])
@pytest.mark.parametrize("dtype,math", [("f32", "x8"), ("f32", "x6h"), ("bf16", None)])
def test_config4_ensemble_vs_fp64(evalset, dtype, math, grouped):
    """grouped=True is evaluate.py's default path (one jr.ensemble.
    EnsembleEngine for every member); per_member is
    --per_member (one jr.Engine each)."""
    import evaluate
    from jr import checkpoint
    data, paths, _ = evalset
    engines = evaluate.make_engines(paths, checkpoint.read_meta(paths[0]), B, dtype=dtype, grouped=grouped,
                                    conv_math=math or "x8")
    tiles = [engines.tiles] if grouped else [e.tiles for e in engines]
    assert all(t == "pinned" for t in tiles), tiles
    preds, labels, ids = evaluate.predict_all(engines, data, B)
    assert ids == list(range(len(ids))) and labels.shape == G["labels"].shape
    assert np.array_equal(labels, G["labels"])
    got = np.stack(preds).astype(np.float64)                  # [M, N, 1]
    want = G["preds"]
    err = np.abs(got - want).max()
    ens = np.mean(np.array(preds), axis=0)                    # evaluate.py:214-217 (float32)
    auc, brier, conf = _metrics(labels, ens)
    print(f"config 4 {dtype} {math}: max |pred - fp64| {err:.2e}, AUC {auc:.6f} vs {float(G['auc']):.6f}, "
          f"Brier {brier:.6f} vs {float(G['brier']):.6f}")
    if dtype == "f32":
        assert err < 1e-4, err
        assert round(auc, 3) == round(float(G["auc"]), 3) and abs(auc - float(G["auc"])) < 5e-4
        assert abs(brier - float(G["brier"])) < 1e-5
        assert np.array_equal(conf, G["confusion"])
    else:   # bars from the emulated-bf16 oracle's own gap to fp64 on the same fixture
        err_emu = np.abs(G["preds_bf16emu"] - want).max()
        auc_emu = abs(float(G["auc_bf16emu"]) - float(G["auc"]))
        brier_emu = abs(float(G["brier_bf16emu"]) - float(G["brier"]))
        print(f"  emulated bf16: max |pred - fp64| {err_emu:.2e}, |AUC gap| {auc_emu:.2e}, |Brier gap| {brier_emu:.2e}")
        assert err <= 3 * err_emu, (err, err_emu)
        # (floors: one sample of an AUC / Brier gap can be ~0)
        assert abs(auc - float(G["auc"])) <= 3 * auc_emu + 2e-3, (auc, auc_emu)
        assert abs(brier - float(G["brier"])) <= 3 * brier_emu + 2e-4, (brier, brier_emu)


def _cli(args, env_extra, cwd, log_dir=None):
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([PKG, ROOT]), **env_extra)
    r = subprocess.run(args, capture_output=True, text=True, env=env, cwd=cwd, timeout=900)
    if r.returncode != 0 and log_dir is not None:     # the ranks' own stderr (torchrun --redirects)
        import glob
        for f in sorted(glob.glob(os.path.join(str(log_dir), "**", "stderr.log"), recursive=True)):
            print(f"---- {f}\n{open(f).read()[-4000:]}")
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    return r.stdout


def test_cli_two_ranks_equal_one_rank(evalset):
    data, paths, d = evalset
    lm = ",".join(paths)
    ev = os.path.join(PKG, "evaluate.py")
    one_csv, two_csv = str(d / "one.csv"), str(d / "two.csv")
    out1 = _cli([sys.executable, ev, "-o", "--data_dir", data, "-lm", lm, "-so", one_csv, "-b", str(B)], {}, str(d))
    port = 29500 + os.getpid() % 1000
    # each rank's stdout to its own file (--redirects): on the shared stream
    # rank 1's gloo connection line could be split by rank 0's output
    logs = d / "torchrun_logs"
    _cli([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
          "--master-addr", "127.0.0.1", "--master-port", str(port), "--log-dir", str(logs), "--redirects", "3",
          ev, "-o", "--data_dir", data, "-lm", lm, "-so", two_csv, "-b", str(B)],
         {"JR_DIST_BACKEND": "gloo", "JR_ONE_DEVICE": "1"}, str(d), log_dir=logs)
    rank0 = list(logs.glob("*/attempt_*/0/stdout.log"))
    assert len(rank0) == 1, rank0
    out2 = rank0[0].read_text()
    # (gloo's own connection log line is not evaluate.py output; blank lines
    # are not compared either)
    strip = lambda s: [ln for ln in s.splitlines() if "Saving operating" not in ln and "amdgpu.ids" not in ln  # noqa: E731
                       and not ln.startswith("[Gloo]") and ln.strip()]
    assert strip(out1) == strip(out2), (out1, out2)
    assert open(one_csv).read() == open(two_csv).read()
    # the default (grouped) CLI against the fp64 fixture: the printed AUC to
    # 3 decimals (north_star) and the confusion matrix at the operating point
    import re
    auc = float(re.search(r"AUC:\s*([0-9.eE+-]+)", out1).group(1))
    assert round(auc, 3) == round(float(G["auc"]), 3), (auc, float(G["auc"]))
    lines = out1.splitlines()
    k = next(i for i, ln in enumerate(lines) if ln.startswith("Confusion matrix"))
    conf = [int(v) for v in re.findall(r"-?\d+", " ".join(lines[k + 1:k + 3]))]
    assert conf == [int(v) for v in np.asarray(G["confusion"]).reshape(-1)], (conf, G["confusion"])
