"""Teacher-forced per-layer parity of the whole Inception-v3 step, fp32 and
bf16, against the fp64 numpy oracle (oracle/tf_ops.py).

Every op of the real network (94 conv2d_bn, 13 pools, GAP, head and the
whole backward) is checked on the ENGINE'S OWN inputs to that op: the
reference conv of layer k reads the engine's activation buffer feeding layer
k, the reference BN reads the engine's raw conv output, the reference
backward of layer k reads the engine's gradient arriving at layer k.  Errors
therefore do not compound through the depth of the net (which amplifies an
input perturbation ~10^3-fold at these small BN populations, see
test_gpu_engine.py), so each op is held to the precision of ONE op:

  fp32: 1e-5 of the output's max |value| (forward), 1e-4 of the gradient's
        norm (backward; sums over B*H*W);
  bf16: operands and outputs are bf16 (8 mantissa bits, 2^-9 relative per
        rounding), products accumulate in fp32: 1.6e-2 of max |value| on the
        bf16 outputs (two roundings: the kernel's and the checker's bf16
        rounding of the raw output it compares against), 2e-2 of the norm for
        gradients that pass through bf16 buffers, 1e-4 for BN statistics.

The test also pins the concat-free slice layout: each branch's output must
land in its channel slice of the block buffer, and the gradient of a buffer
read by several layers must equal the SUM of their contributions.
"""
import numpy as np
import pytest

from oracle import tf_ops as R

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

TOL = {
    "f32": dict(raw=1e-5, act=1e-5, stats=1e-5, pool=1e-6, grad=1e-4, dx=1e-4, head=1e-5),
    "bf16": dict(raw=8e-3, act=1.6e-2, stats=1e-4, pool=8e-3, grad=2e-2, dx=2e-2, head=1e-4),
}


def _f64(t):
    return t.detach().float().cpu().numpy().astype(np.float64)


def _bf16(a):
    return torch.as_tensor(np.asarray(a, np.float32)).to(torch.bfloat16).double().numpy()


def _maxrel(got, ref):
    return float(np.max(np.abs(got - ref)) / max(np.max(np.abs(ref)), 1e-30))


def _normrel(got, ref):
    return float(np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30))


@pytest.mark.parametrize("dtype,res,batch", [("f32", 107, 3), ("f32x8", 107, 3), ("bf16", 107, 3), ("bf16", 139, 4)])
def test_every_layer_teacher_forced(dtype, res, batch):
    from jr.engine import Engine
    from jr.init import unflatten
    from jr import synth

    tol = TOL["f32" if dtype == "f32x8" else dtype]      # x8 is held to the fp32 tolerances
    # (fuse_pool=False: every activation buffer materialised for the per-layer
    # checks; the fused BN + max-pool is bitwise the pair, test_gpu_engine.py)
    eng = Engine(batch, res, res, seed=7, dtype="f32" if dtype == "f32x8" else dtype,
                 conv_math={"f32": "f32", "f32x8": "x8"}.get(dtype), fuse_pool=False)
    imgs = synth.fundus_batch(3, batch, res)
    y = np.array([[1.0], [0.0], [1.0], [0.0]][:batch], np.float32)
    eng.set_batch(imgs, y)
    eng.forward()
    eng.backward()
    eng.synchronize()
    g, B = eng.g, batch
    P = unflatten(g, eng.params_numpy())
    G = unflatten(g, eng.grads_numpy())
    rnd = _bf16 if dtype == "bf16" else (lambda a: np.asarray(a, np.float64))

    def buf(bid, dacts=False):
        b = g.bufs[bid]
        t = (eng.dacts if dacts else eng.acts)[bid]
        c = eng.in_stride if (bid == g.input_buf and not dacts) else b.c
        return _f64(t).reshape(B, b.h, b.w, c)

    acts = {b.id: buf(b.id) for b in g.bufs}
    acts[g.input_buf] = acts[g.input_buf][..., :g.bufs[g.input_buf].c]
    # the engine's image equals convert_image_dtype (rounded to the path dtype)
    assert np.array_equal(acts[g.input_buf], rnd(R.convert_image_dtype_u8(imgs)))
    dacts = {b.id: buf(b.id, True) for b in g.bufs if b.id != g.input_buf}
    dx_ref = {bid: np.zeros_like(v) for bid, v in dacts.items()}
    bad = []

    def check(what, err, lim):
        if not err <= lim:
            bad.append((what, err, lim))

    # ------------------------------------------------------------- forward
    for i, n in enumerate(g.nodes):
        x = acts[n.x]
        yb = acts[n.y.buf][..., n.y.c_off:n.y.c_off + (n.cout if n.kind == "conv" else n.c)]
        if n.kind == "conv":
            W = rnd(P[f"{n.name}/kernel"])
            raw = R.conv2d(x, W, n.stride, n.padding)
            raw_e = _f64(eng.raw[n.idx]).reshape(raw.shape)
            check(f"{n.name} raw", _maxrel(raw_e, raw), tol["raw"])
            beta = P[f"batch_normalization_{n.idx + 1}/beta"].astype(np.float64)
            y_ref, mean, invstd = R.bn_relu_fwd(raw_e, beta)
            check(f"{n.name} mean", float(np.max(np.abs(_f64(eng.mean[n.idx]) - mean)) /
                                          max(np.max(np.abs(raw_e)), 1e-30)), tol["stats"])
            check(f"{n.name} invstd", _maxrel(_f64(eng.invstd[n.idx]), invstd), tol["stats"])
            check(f"{n.name} bn_relu", _maxrel(yb, y_ref), tol["act"])
        elif n.kind == "maxpool":
            y_ref, am = R.maxpool3x3s2(x)
            check(f"maxpool{i}", _maxrel(yb, y_ref), 0.0)
            am_e = eng.argmax[i].cpu().numpy().reshape(am.shape)
            # ties only occur among ReLU zeros, whose gradient is masked anyway
            check(f"maxpool{i} argmax", float(np.mean((am_e != am) & (y_ref > 0))), 0.0)
        else:
            check(f"avgpool{i}", _maxrel(yb, R.avgpool3x3s1_same(x)), tol["pool"])
    ob = g.bufs[g.output_buf]
    feat = eng.feat.cpu().numpy().astype(np.float64).reshape(B, ob.c)
    check("gap", _maxrel(feat, R.global_avg_pool(acts[g.output_buf])), tol["head"])
    logits = eng.logits.cpu().numpy().astype(np.float64)[:B].reshape(B, 1)
    z = R.dense(feat, P["dense/kernel"].astype(np.float64), P["dense/bias"].astype(np.float64))
    check("logits", _maxrel(logits, z), tol["head"])

    # ------------------------------------------------------------- backward
    dz = R.sigmoid_xent_grad(z, y.astype(np.float64))
    check("dense/kernel grad", _normrel(G["dense/kernel"], feat.T @ dz), tol["head"] * 10)
    dfeat = dz @ P["dense/kernel"].astype(np.float64).T
    dx_ref[g.output_buf] += np.broadcast_to((dfeat / (ob.h * ob.w))[:, None, None, :], dx_ref[g.output_buf].shape)
    for i in range(len(g.nodes) - 1, -1, -1):
        n = g.nodes[i]
        c = n.cout if n.kind == "conv" else n.c
        dy = dacts[n.y.buf][..., n.y.c_off:n.y.c_off + c]
        if n.kind == "conv":
            x = acts[n.x]
            raw_e = _f64(eng.raw[n.idx]).reshape(B, n.ho, n.wo, n.cout)
            beta = P[f"batch_normalization_{n.idx + 1}/beta"].astype(np.float64)
            mask = acts[n.y.buf][..., n.y.c_off:n.y.c_off + c] > 0
            draw, dbeta = R.bn_relu_bwd(dy, raw_e, beta, mask=mask)
            check(f"{n.name} dbeta", _normrel(G[f"batch_normalization_{n.idx + 1}/beta"], dbeta), tol["grad"])
            draw_r = rnd(draw)
            dW = R.conv2d_bwd_filter(x, draw_r, P[f"{n.name}/kernel"].shape, n.stride, n.padding)
            check(f"{n.name} dW", _normrel(G[f"{n.name}/kernel"], dW), tol["grad"])
            if n.x != g.input_buf:
                W = rnd(P[f"{n.name}/kernel"])
                dx_ref[n.x] += R.conv2d_bwd_data(draw_r, W, x.shape, n.stride, n.padding)
        elif n.kind == "maxpool":
            am = eng.argmax[i].cpu().numpy().reshape(B, n.ho, n.wo, n.c)
            dx_ref[n.x] += R.maxpool3x3s2_bwd(dy, am, acts[n.x].shape)
        else:
            dx_ref[n.x] += R.avgpool3x3s1_same_bwd(dy)
        # every consumer of buffer n.x has run once the producer's turn comes
    for bid, ref in dx_ref.items():
        check(f"d[{g.bufs[bid].name}]", _normrel(dacts[bid], ref), tol["dx"])
    assert not bad, f"{len(bad)} checks failed, first: {bad[:8]}"
