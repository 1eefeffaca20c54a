"""Generate the committed golden fixtures under tests/golden/ (TEST ORACLE).

Parity status: UNPINNED — the reference (TF 1.x) cannot run here and ships no
vectors (oracle/__init__.py).  These fixtures freeze the oracle's own outputs
(numpy fp64 per op, torch-CPU fp64 for the whole network) so that
  * CPU tests can check the oracle against them (regression, and the torch
    cross-formulation), and
  * GPU tests on the box (where /root/reference and this generator's time
    budget are absent) compare libjr against fixed expected values.
Weights are NOT stored: they are regenerated from the seed by jr.init
(numpy PCG64), inputs from jr.synth (PCG64(432 + i)).

  python oracle/make_golden.py [--only ops,metrics,net107,net299,curve,curve16,curve16bf,net299b64,net587b2,eval299,curve16bf32]

BASELINE-size fixtures (net299b64: configs 2-3 geometry, 299^2 B=64;
net587b2: config 5 geometry, 587^2 B=2) hold the fp64 results AND the same
step by the fp32 CPU restatement ("*_fp32" keys): the fp32-vs-fp64 gap of an
independent fp32 implementation is the envelope the GPU tests scale.  Per
gradient tensor they keep its norm and its projection on a seeded
Rademacher vector (grad_proj, seed 1000 + index in grad_names): a norm
misses a permuted or sign-flipped gradient, the projection does not.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "jama16-retina-replication_amd"))
OUT = os.path.join(ROOT, "tests", "golden")

from oracle import metrics_ref as MR  # noqa: E402
from oracle import tf_ops as R  # noqa: E402

CONV_GOLDEN = [  # n, h, w, cin, cout, kh, kw, stride, padding
    (2, 9, 9, 8, 16, 3, 3, 1, "same"),
    (2, 11, 11, 8, 16, 3, 3, 2, "valid"),
    (1, 7, 8, 4, 16, 1, 7, 1, "same"),
    (1, 8, 7, 4, 16, 7, 1, 1, "same"),
    (2, 9, 9, 3, 16, 3, 3, 2, "valid"),
    (1, 6, 6, 12, 16, 5, 5, 1, "same"),
]


def ops():
    rng = np.random.default_rng(20261015)
    d = {}
    for i, (n, h, w, ci, co, kh, kw, s, p) in enumerate(CONV_GOLDEN):
        x = rng.standard_normal((n, h, w, ci)).astype(np.float32)
        wt = (rng.standard_normal((kh, kw, ci, co)) / np.sqrt(kh * kw * ci)).astype(np.float32)
        y = R.conv2d(x, wt, s, p)
        dy = rng.standard_normal(y.shape).astype(np.float32)
        d[f"conv{i}_x"], d[f"conv{i}_w"], d[f"conv{i}_dy"] = x, wt, dy
        d[f"conv{i}_y"] = y
        d[f"conv{i}_dx"] = R.conv2d_bwd_data(dy, wt, x.shape, s, p)
        d[f"conv{i}_dw"] = R.conv2d_bwd_filter(x, dy, wt.shape, s, p)
    x = (rng.standard_normal((3, 5, 5, 8)) * 2 + 1).astype(np.float32)
    beta = rng.standard_normal(8).astype(np.float32) * 0.3
    dy = rng.standard_normal(x.shape).astype(np.float32)
    d["bn_x"], d["bn_beta"], d["bn_dy"] = x, beta, dy
    d["bn_y"], d["bn_mean"], d["bn_invstd"] = R.bn_relu_fwd(x, beta)
    d["bn_dx"], d["bn_dbeta"] = R.bn_relu_bwd(dy, x, beta)
    x = np.maximum(rng.standard_normal((2, 9, 11, 4)), 0).astype(np.float32)
    d["mp_x"] = x
    d["mp_y"], d["mp_arg"] = R.maxpool3x3s2(x)
    d["mp_dy"] = rng.standard_normal(d["mp_y"].shape).astype(np.float32)
    d["mp_dx"] = R.maxpool3x3s2_bwd(d["mp_dy"], d["mp_arg"], x.shape)
    x = rng.standard_normal((2, 4, 6, 4)).astype(np.float32)
    d["ap_x"], d["ap_y"] = x, R.avgpool3x3s1_same(x)
    d["ap_dy"] = rng.standard_normal(x.shape).astype(np.float32)
    d["ap_dx"] = R.avgpool3x3s1_same_bwd(d["ap_dy"])
    f = rng.standard_normal((6, 16)).astype(np.float32)
    W = rng.standard_normal((16, 1)).astype(np.float32) * 0.3
    b = np.array([0.2], np.float32)
    y = (rng.random((6, 1)) < 0.4).astype(np.float32)
    z = R.dense(f, W, b)
    d.update(head_f=f, head_w=W, head_b=b, head_y=y, head_z=z, head_p=R.sigmoid(z),
             head_loss=np.array(R.sigmoid_xent_mean(z, y)), head_dz=R.sigmoid_xent_grad(z, y))
    w0, g0, a0 = (rng.standard_normal(10).astype(np.float32) for _ in range(3))
    w1, a1 = R.nesterov(w0.astype(np.float64), g0, a0)
    d.update(nest_w=w0, nest_g=g0, nest_a=a0, nest_w1=w1, nest_a1=a1)
    u8 = np.arange(256, dtype=np.uint8)
    d["u8"], d["u8_scaled"] = u8, R.convert_image_dtype_u8(u8)
    np.savez_compressed(os.path.join(OUT, "ops_small.npz"), **d)


def metrics():
    rng = np.random.default_rng(7)
    n = 1000
    y = (rng.random((n, 1)) < 0.3).astype(np.float32)
    p = np.clip(0.5 * rng.random((n, 1)) + 0.4 * y, 0, 1).astype(np.float32)
    thr = MR.generate_thresholds(200, 1e-7) + [0.5]
    tp, fp, fn, tn = MR.counts_at_thresholds(y, p, thr)
    spec, sens = MR.spec_sens(tp, fp, fn, tn)
    np.savez_compressed(os.path.join(OUT, "metrics.npz"), labels=y, preds=p, thresholds=np.array(thr),
                        tp=tp, fp=fp, fn=fn, tn=tn, spec=spec, sens=sens,
                        auc=np.array(MR.auc(y, p)), brier=np.array(MR.brier(y, p)),
                        confusion=MR.confusion_matrix(tp[-1], fp[-1], fn[-1], tn[-1]))


def grad_projection(g, i):
    """<g, r_i> for the seeded Rademacher vector r_i (seed 1000 + i)."""
    r = np.random.default_rng(1000 + i).integers(0, 2, g.size, dtype=np.int8).astype(np.float64) * 2 - 1
    return float(np.dot(np.asarray(g, np.float64).ravel(), r))


def _net(res, batch, seed, steps=1, cycle=None, dtype="float64", proj=False, bf16=False, order_seed=None,
         threads=None):
    import torch
    from jr import synth
    from jr.inception import build_inception_v3
    from jr.init import init_params, unflatten
    from oracle.inception_ref import InceptionV3Ref
    torch.set_num_threads(threads or os.cpu_count() or 8)
    g = build_inception_v3(res, res)
    ref = InceptionV3Ref(unflatten(g, init_params(g, seed)), getattr(torch, dtype), emulate_bf16=bf16,
                         order_seed=order_seed)
    pool = cycle or batch
    imgs = synth.fundus_batch(0, pool, res)
    labels = synth.labels(0, pool)
    state, losses = {}, []
    out = {}
    for step in range(steps):
        k = (step * batch) % pool
        x = imgs[k:k + batch].astype(np.float32) * np.float32(1 / 255)
        y = labels[k:k + batch]
        loss, probs, grads = ref.train_step(x, y, state)
        losses.append(loss)
        if step == 0:
            out["logits"] = ref.last_logits
            out["probs"] = probs
            out["loss0"] = np.array(loss)
            names = sorted(grads)
            out["grad_names"] = np.array(names)
            out["grad_norms"] = np.array([np.linalg.norm(grads[k_]) for k_ in names])
            if proj:
                out["grad_proj"] = np.array([grad_projection(grads[k_], i) for i, k_ in enumerate(names)])
            del grads
    out["losses"] = np.array(losses)
    out.update(res=np.array(res), batch=np.array(batch), seed=np.array(seed), pool=np.array(pool))
    return out


EVAL299 = dict(n=280, res=299, batch=32, members=3, p=0.3, start=5000, label_seed=11)


def eval_records(out_dir: str) -> None:
    """The config-4 test set of the eval299b32 fixture: 280 synthetic fundus
    images (299^2, JPEG q=100, labels Bernoulli(0.3)), ONE shard (the
    reference lists shards in os.listdir order, lib/dataset.py:5-8, so one
    shard keeps the record order fixed), as the GPU test rewrites it."""
    from jr import synth_records
    e = EVAL299
    synth_records.write_split(out_dir, e["n"], e["res"], p=e["p"], start=e["start"], num_shards=1, name="test",
                              label_seed=e["label_seed"])


def eval_batches(data_dir: str, batch: int):
    """(uint8 batches, label batches, sha256 of every decoded pixel) as
    evaluate.predict_all reads them (lib.dataset, native decode, IFAST)."""
    import hashlib
    import lib.dataset as D
    ds = D.initialize_dataset(data_dir, batch, num_workers=8, prefetch_buffer_size=2 * batch,
                              image_data_format="channels_last", num_channels=3, image_dim=[299, 299],
                              decode_dtype="uint8")
    xs, ys, h = [], [], hashlib.sha256()
    it = iter(ds)
    try:
        for x, y in it:
            xs.append(np.array(x))
            ys.append(np.array(y))
            h.update(np.ascontiguousarray(xs[-1]).tobytes())
    finally:
        D.close_iterator(it)
    return xs, ys, h.hexdigest()


def eval299():
    """BASELINE config 4 at its workload geometry:
    evaluate.py -lm of 3 members (Keras init seeds 0-2) over 280 test images
    at 299^2 in eval batches of 32 (the last one partial, 24), batch-statistics
    BN per batch (App. C Q1).  fp64 oracle predictions per member, the linear
    ensemble mean (evaluate.py:214-217) and its TF metrics (200-threshold AUC,
    Brier, confusion and spec/sens at the 0.5 operating threshold)."""
    import tempfile
    import torch
    from jr.inception import build_inception_v3
    from jr.init import init_params, unflatten
    from oracle.inception_ref import InceptionV3Ref
    torch.set_num_threads(os.cpu_count() or 8)
    e = EVAL299
    with tempfile.TemporaryDirectory() as d:
        eval_records(d)
        xs, ys, digest = eval_batches(d, e["batch"])
    g = build_inception_v3(e["res"], e["res"])
    preds, preds_bf = [], []
    for m in range(e["members"]):
        for bf, out in ((False, preds), (True, preds_bf)):
            # fp64, and the same forward with bf16 storage emulated where the
            # GPU bf16 path stores bf16 (an independent bf16 implementation:
            # its gap to fp64 is the envelope the bf16 engine is judged by)
            ref = InceptionV3Ref(unflatten(g, init_params(g, m)), torch.float64, requires_grad=False,
                                 emulate_bf16=bf)
            pm = []
            for x in xs:
                with torch.no_grad():
                    _, p, _ = ref.forward(x.astype(np.float32) * np.float32(1 / 255))
                pm.append(np.asarray(p, np.float64).reshape(-1, 1))
            out.append(np.vstack(pm))
        print(f"eval299 member {m} done", flush=True)
    preds = np.stack(preds)                           # [M, N, 1] fp64
    preds_bf = np.stack(preds_bf)
    labels = np.vstack(ys).astype(np.float32)
    ens = preds.astype(np.float32).mean(axis=0)       # evaluate.py: np.mean of float32 predictions
    thr = MR.generate_thresholds(200, 1e-7) + [0.5]
    tp, fp, fn, tn = MR.counts_at_thresholds(labels, ens, thr)
    spec, sens = MR.spec_sens(tp, fp, fn, tn)
    ens_bf = preds_bf.astype(np.float32).mean(axis=0)
    np.savez_compressed(os.path.join(OUT, "eval_res299_b32.npz"), preds=preds, labels=labels, ens=ens,
                        preds_bf16emu=preds_bf, auc_bf16emu=np.array(MR.auc(labels, ens_bf)),
                        brier_bf16emu=np.array(MR.brier(labels, ens_bf)),
                        input_sha256=np.array(digest), auc=np.array(MR.auc(labels, ens)),
                        brier=np.array(MR.brier(labels, ens)), confusion=MR.confusion_matrix(tp[-1], fp[-1], fn[-1],
                                                                                             tn[-1]),
                        spec=spec, sens=sens, **{k: np.array(v) for k, v in e.items()})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="ops,metrics,net107,net299,curve")
    a = ap.parse_args()
    os.makedirs(OUT, exist_ok=True)
    todo = a.only.split(",")
    t0 = time.time()
    if "ops" in todo:
        ops()
    if "metrics" in todo:
        metrics()
    if "net107" in todo:
        np.savez_compressed(os.path.join(OUT, "net_res107_b3.npz"), **_net(107, 3, 1))
    if "net299" in todo:
        np.savez_compressed(os.path.join(OUT, "net_res299_b4.npz"), **_net(299, 4, 0))
    if "curve" in todo:
        # 100 Nesterov steps at B=4, 299^2, fixed unshuffled stream of 8 images
        # plus the same run in fp32 on the CPU: B=4 batch-stat BN with momentum
        # amplifies fp32 round-off within a few steps, so the fp32-vs-fp64
        # gap is the envelope any fp32 implementation is judged against
        curve = _net(299, 4, 0, steps=100, cycle=8)
        curve["losses_fp32_cpu"] = _net(299, 4, 0, steps=100, cycle=8, dtype="float32")["losses"]
        np.savez_compressed(os.path.join(OUT, "loss_curve_res299_b4.npz"), **curve)
    if "curve16" in todo:
        # 100 Nesterov steps at B=16, 299^2, fixed unshuffled stream of 32
        # images (two alternating batches), fp64 and fp32 CPU: per-step
        # tracking fixture (BN populations 16x larger than the B=4 curve)
        curve = _net(299, 16, 0, steps=100, cycle=32)
        curve["losses_fp32_cpu"] = _net(299, 16, 0, steps=100, cycle=32, dtype="float32")["losses"]
        np.savez_compressed(os.path.join(OUT, "loss_curve_res299_b16.npz"), **curve)
        print(f"curve16: {time.time() - t0:.0f}s", flush=True)
    if "curve16bf" in todo:
        # the same 100 steps by the oracle with bf16 storage emulated where the
        # GPU bf16 path stores bf16 (an independent bf16 implementation): its
        # gap to fp64 is the envelope the bf16 engine's curve is judged by
        p = os.path.join(OUT, "loss_curve_res299_b16.npz")
        curve = dict(np.load(p))
        curve["losses_bf16emu"] = _net(299, 16, 0, steps=100, cycle=32, bf16=True)["losses"]
        np.savez_compressed(p, **curve)
        print(f"curve16bf: {time.time() - t0:.0f}s", flush=True)
    if "curve16bf32" in todo:
        # a SECOND independent bf16 implementation of the same 100 steps: bf16
        # storage emulated as above but every product summed in fp32 (the
        # GPU's accumulation precision) instead of fp64.  The spread between
        # the two emulations calibrates the bf16 curve test's per-step bar
        #  without reference to any GPU run.
        p = os.path.join(OUT, "loss_curve_res299_b16.npz")
        curve = dict(np.load(p))
        curve["losses_bf16emu32"] = _net(299, 16, 0, steps=100, cycle=32, dtype="float32", bf16=True)["losses"]
        np.savez_compressed(p, **curve)
        print(f"curve16bf32: {time.time() - t0:.0f}s", flush=True)
    for key, batch, cycle in (("curvecal4", 4, 8), ("curvecal16", 16, 32)):
        if key not in todo:
            continue
        # K independent fp32 samples of the same 100 steps:
        # each with its own fp32-exact summation order (permuted conv input
        # channels and batch order, order seeds 1..K) and thread count; their
        # spread around fp64 calibrates the fp32 curve test's bars
        p = os.path.join(OUT, f"loss_curve_res299_b{batch}.npz")
        curve = dict(np.load(p))
        K = int(os.environ.get("CURVECAL_K", "6"))
        threads = [8, 4, 2, 8, 6, 3, 8, 5][:K]
        cal = [_net(299, batch, 0, steps=100, cycle=cycle, dtype="float32", order_seed=k + 1,
                    threads=threads[k % len(threads)])["losses"] for k in range(K)]
        curve["losses_fp32_cal"] = np.stack(cal)
        curve["losses_fp32_cal_threads"] = np.array([threads[k % len(threads)] for k in range(K)])
        np.savez_compressed(p, **curve)
        print(f"{key}: {time.time() - t0:.0f}s", flush=True)
    if "eval299" in todo:
        eval299()
        print(f"eval299: {time.time() - t0:.0f}s", flush=True)
    for key, res, batch in (("net299b64", 299, 64), ("net587b2", 587, 2)):
        if key in todo:
            d = _net(res, batch, 0, proj=True)
            d32 = _net(res, batch, 0, dtype="float32", proj=True)
            dbf = _net(res, batch, 0, proj=True, bf16=True)
            for k_ in ("logits", "probs", "loss0", "grad_norms", "grad_proj"):
                d[k_ + "_fp32"] = d32[k_]
                d[k_ + "_bf16emu"] = dbf[k_]
            np.savez_compressed(os.path.join(OUT, f"net_res{res}_b{batch}.npz"), **d)
            print(f"{key}: {time.time() - t0:.0f}s", flush=True)
    print(f"golden fixtures written to {OUT} in {time.time() - t0:.0f}s")


if __name__ == "__main__":
    main()
