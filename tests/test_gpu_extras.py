"""north_star extras beyond the reference's own graph, through the C-ABI:

* softmax cross-entropy head (jr_head_fwd/bwd mode JR_HEAD_SOFTMAX) vs the
  fp64 oracle (oracle/tf_ops.softmax_xent_mean): logits / dfeat / dW / db
  within 1e-5 of max|ref|, probs and loss within 1e-6;
* the optimizers vs IEEE fp32 restatements in TF's operation order
  (oracle/tf_ops: ApplyMomentum with and without Nesterov, ApplyAdam):
  every kernel writes its expression with correctly rounded _rn ops in that
  order, so the results are BITWISE the numpy float32 evaluation, step after
  step (several steps, so state bugs show);
* Adam and plain momentum wired through the Engine (optimizer='adam' /
  'momentum'): one training step's update equals the restatement applied to
  the engine's own gradient, bitwise.
"""
import ctypes

import numpy as np
import pytest

from oracle import tf_ops as R

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

_KEEP = []


@pytest.fixture(autouse=True)
def _keep_alive():
    yield
    torch.cuda.synchronize()
    _KEEP.clear()


def _lib():
    from jr import _ffi
    _ffi.init(0)
    return _ffi


def dev(a):
    t = torch.as_tensor(np.ascontiguousarray(a, np.float32)).cuda()
    _KEEP.append(t)
    return t


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def relerr(got, ref):
    ref = np.asarray(ref, np.float64)
    return float(np.max(np.abs(got - ref)) / max(np.max(np.abs(ref)), 1e-30))


@pytest.mark.parametrize("n,c,units", [(6, 64, 5), (32, 2048, 2), (3, 2048, 16)])
def test_softmax_head(n, c, units):
    ffi = _lib()
    L = ffi.load()
    rng = np.random.default_rng(n * units)
    f = np.maximum(rng.standard_normal((n, c)), 0).astype(np.float32)
    W = (rng.standard_normal((c, units)) * 0.05).astype(np.float32)
    b = (rng.standard_normal(units) * 0.1).astype(np.float32)
    y = np.eye(units, dtype=np.float32)[rng.integers(0, units, n)]
    F, Wd, Bd, Y = dev(f), dev(W), dev(b), dev(y)
    LOG, PR, LOSS = (torch.zeros(n * units, device="cuda") for _ in range(2)), None, None
    LOG, PR = torch.zeros(n * units, device="cuda"), torch.zeros(n * units, device="cuda")
    LOSS = torch.zeros(1, device="cuda")
    ffi.check("head", L.jr_head_fwd(1, F.data_ptr(), Wd.data_ptr(), Bd.data_ptr(), Y.data_ptr(), n, c, units,
                                    LOG.data_ptr(), PR.data_ptr(), LOSS.data_ptr(), None))
    z = R.dense(f, W, b)
    loss, p, dz = R.softmax_xent_mean(z, y)
    assert relerr(host(LOG).reshape(n, units), z) < 1e-5
    assert np.max(np.abs(host(PR).reshape(n, units) - p)) < 1e-6
    assert abs(float(host(LOSS)[0]) - loss) < 1e-6 * max(1.0, loss)
    DF, DW, DB = torch.zeros(n * c, device="cuda"), torch.zeros(c * units, device="cuda"), torch.zeros(units, device="cuda")
    ffi.check("head bwd", L.jr_head_bwd(1, F.data_ptr(), Wd.data_ptr(), PR.data_ptr(), Y.data_ptr(), n, c, units,
                                        DF.data_ptr(), DW.data_ptr(), DB.data_ptr(), None))
    assert relerr(host(DW).reshape(c, units), f.T.astype(np.float64) @ dz) < 1e-5
    assert relerr(host(DB), dz.sum(0)) < 1e-5
    assert relerr(host(DF).reshape(n, c), dz @ W.T.astype(np.float64)) < 1e-5


def _f32(*a):
    return [np.asarray(x, np.float32) for x in a]


def test_optimizers_bitwise_tf_order():
    ffi = _lib()
    L = ffi.load()
    rng = np.random.default_rng(3)
    n = 10007                                            # float4 body + scalar tail
    w0 = rng.standard_normal(n).astype(np.float32)
    gs = [rng.standard_normal(n).astype(np.float32) for _ in range(4)]
    f = np.float32
    # Nesterov / momentum / SGD, 4 steps each
    for kind in ("nesterov", "momentum", "sgd"):
        W, A = dev(w0), dev(np.zeros(n))
        w, a = _f32(w0, np.zeros(n))
        for g in gs:
            G = dev(g)
            if kind == "nesterov":
                ffi.check(kind, L.jr_nesterov_update(W.data_ptr(), G.data_ptr(), A.data_ptr(), n, 3e-3, 0.9, 1.0, None))
                a = a * f(0.9) + g
                w = w - (g * f(3e-3) + a * f(0.9) * f(3e-3))
            elif kind == "momentum":
                ffi.check(kind, L.jr_momentum_update(W.data_ptr(), G.data_ptr(), A.data_ptr(), n, 3e-3, 0.9, 1.0, None))
                w, a = _f32(*R.momentum(w, g, a, f(3e-3), f(0.9)))
            else:
                ffi.check(kind, L.jr_sgd_update(W.data_ptr(), G.data_ptr(), n, 3e-3, 1.0, None))
                w = w - g * f(3e-3)
        assert np.array_equal(host(W), w), kind
        if kind != "sgd":
            assert np.array_equal(host(A), a), kind
    # Adam, 4 steps
    W, M, V = dev(w0), dev(np.zeros(n)), dev(np.zeros(n))
    w, m, v = _f32(w0, np.zeros(n), np.zeros(n))
    for t, g in enumerate(gs, 1):
        w, m, v, alpha = R.adam_f32(w, g, m, v, t, lr=1e-3)
        G = dev(g)
        ffi.check("adam", L.jr_adam_update(W.data_ptr(), G.data_ptr(), M.data_ptr(), V.data_ptr(), n, float(alpha),
                                           0.9, 0.999, 1e-8, 1.0, None))
        assert np.array_equal(host(M), m) and np.array_equal(host(V), v), t
        assert np.array_equal(host(W), w), t


@pytest.mark.parametrize("opt", ["adam", "momentum"])
def test_engine_optimizer_step(opt):
    """Engine(optimizer=...) applies the restated update to its own gradient."""
    from jr.engine import Engine
    from jr import synth
    eng = Engine(2, 107, 107, seed=4, optimizer=opt, lr=1e-3 if opt == "adam" else 3e-3, autotune=False)
    eng.set_batch(synth.fundus_batch(0, 2, 107), np.array([[1.0], [0.0]], np.float32))
    w = eng.params.cpu().numpy().copy()
    m = np.zeros_like(w)
    v = np.zeros_like(w)
    for t in (1, 2):
        eng.forward()
        eng.backward()
        eng.synchronize()            # the engine's lane streams, not torch's current stream
        g = eng.grads.cpu().numpy().copy()
        eng.apply_update()
        eng.synchronize()
        if opt == "adam":
            w, m, v, _ = R.adam_f32(w, g, m, v, t, lr=1e-3)
        else:
            w, m = _f32(*R.momentum(w, g, m, np.float32(3e-3), np.float32(0.9)))
        assert np.array_equal(eng.params.cpu().numpy(), w), (opt, t)
