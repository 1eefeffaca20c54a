"""The CPU oracle (test infrastructure) against its committed golden vectors
and against independent formulations.  Parity with TF itself is UNPINNED
(oracle/__init__.py): these checks pin the restatement, not TF."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import metrics_ref as MR
from oracle import tf_ops as R
from oracle.make_golden import CONV_GOLDEN


@pytest.fixture(scope="module")
def ops():
    return np.load(os.path.join(GOLDEN, "ops_small.npz"))


def test_conv_ops_match_golden(ops):
    for i, (n, h, w, ci, co, kh, kw, s, p) in enumerate(CONV_GOLDEN):
        x, wt, dy = ops[f"conv{i}_x"], ops[f"conv{i}_w"], ops[f"conv{i}_dy"]
        np.testing.assert_allclose(R.conv2d(x, wt, s, p), ops[f"conv{i}_y"], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(R.conv2d_bwd_data(dy, wt, x.shape, s, p), ops[f"conv{i}_dx"], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(R.conv2d_bwd_filter(x, dy, wt.shape, s, p), ops[f"conv{i}_dw"], rtol=1e-12,
                                   atol=1e-12)


def test_conv_against_torch_and_autograd(ops):
    """Independent formulation: torch conv2d (NCHW) forward and autograd."""
    torch = pytest.importorskip("torch")
    F = torch.nn.functional
    for i, (n, h, w, ci, co, kh, kw, s, p) in enumerate(CONV_GOLDEN):
        x = torch.tensor(ops[f"conv{i}_x"], dtype=torch.float64).permute(0, 3, 1, 2).requires_grad_()
        wt = torch.tensor(ops[f"conv{i}_w"], dtype=torch.float64).permute(3, 2, 0, 1).requires_grad_()
        pad = ((kh - 1) // 2, (kw - 1) // 2) if p == "same" else (0, 0)
        y = F.conv2d(x, wt, stride=s, padding=pad)
        np.testing.assert_allclose(y.permute(0, 2, 3, 1).detach().numpy(), ops[f"conv{i}_y"], rtol=1e-10, atol=1e-10)
        y.backward(torch.tensor(ops[f"conv{i}_dy"], dtype=torch.float64).permute(0, 3, 1, 2))
        np.testing.assert_allclose(x.grad.permute(0, 2, 3, 1).numpy(), ops[f"conv{i}_dx"], rtol=1e-10, atol=1e-10)
        np.testing.assert_allclose(wt.grad.permute(2, 3, 1, 0).numpy(), ops[f"conv{i}_dw"], rtol=1e-10, atol=1e-10)


def test_bn_relu_against_autograd(ops):
    torch = pytest.importorskip("torch")
    x = torch.tensor(ops["bn_x"], dtype=torch.float64, requires_grad=True)
    beta = torch.tensor(ops["bn_beta"], dtype=torch.float64, requires_grad=True)
    mean = x.mean(dim=(0, 1, 2))
    var = ((x - mean) ** 2).mean(dim=(0, 1, 2))
    y = torch.relu((x - mean) / torch.sqrt(var + 1e-3) + beta)
    np.testing.assert_allclose(y.detach().numpy(), ops["bn_y"], rtol=1e-12, atol=1e-12)
    y.backward(torch.tensor(ops["bn_dy"], dtype=torch.float64))
    np.testing.assert_allclose(x.grad.numpy(), ops["bn_dx"], rtol=1e-9, atol=1e-10)
    np.testing.assert_allclose(beta.grad.numpy(), ops["bn_dbeta"], rtol=1e-12, atol=1e-12)
    y2, m2, i2 = R.bn_relu_fwd(ops["bn_x"], ops["bn_beta"])
    np.testing.assert_allclose(y2, ops["bn_y"], rtol=1e-12)


def test_pools_against_torch(ops):
    torch = pytest.importorskip("torch")
    F = torch.nn.functional
    x = torch.tensor(ops["mp_x"], dtype=torch.float64).permute(0, 3, 1, 2)
    np.testing.assert_array_equal(F.max_pool2d(x, 3, 2).permute(0, 2, 3, 1).numpy(), ops["mp_y"])
    y, arg = R.maxpool3x3s2(ops["mp_x"])
    np.testing.assert_array_equal(arg, ops["mp_arg"])
    np.testing.assert_allclose(R.maxpool3x3s2_bwd(ops["mp_dy"], arg, ops["mp_x"].shape), ops["mp_dx"])
    xa = torch.tensor(ops["ap_x"], dtype=torch.float64).permute(0, 3, 1, 2).requires_grad_()
    ya = F.avg_pool2d(xa, 3, 1, padding=1, count_include_pad=False)      # TF exclude-pad divisor
    np.testing.assert_allclose(ya.permute(0, 2, 3, 1).detach().numpy(), ops["ap_y"], rtol=1e-12)
    ya.backward(torch.tensor(ops["ap_dy"], dtype=torch.float64).permute(0, 3, 1, 2))
    np.testing.assert_allclose(xa.grad.permute(0, 2, 3, 1).numpy(), ops["ap_dx"], rtol=1e-12)


def test_head_loss_optimizer(ops):
    z = R.dense(ops["head_f"], ops["head_w"], ops["head_b"])
    np.testing.assert_allclose(z, ops["head_z"], rtol=1e-12)
    assert abs(R.sigmoid_xent_mean(z, ops["head_y"]) - float(ops["head_loss"])) < 1e-12
    # sigmoid xent equals the naive -y log p - (1-y) log(1-p)
    p = R.sigmoid(z)
    y = ops["head_y"]
    naive = np.mean(-y * np.log(p) - (1 - y) * np.log(1 - p))
    assert abs(naive - float(ops["head_loss"])) < 1e-12
    # finite-difference check of d loss / d z
    eps = 1e-6
    g = np.zeros_like(z)
    for k in range(z.size):
        zp, zm = z.copy(), z.copy()
        zp.flat[k] += eps
        zm.flat[k] -= eps
        g.flat[k] = (R.sigmoid_xent_mean(zp, y) - R.sigmoid_xent_mean(zm, y)) / (2 * eps)
    np.testing.assert_allclose(g, ops["head_dz"], rtol=1e-6, atol=1e-9)
    w1, a1 = R.nesterov(ops["nest_w"].astype(np.float64), ops["nest_g"], ops["nest_a"])
    np.testing.assert_allclose(w1, ops["nest_w1"])
    # TF ApplyMomentum(use_nesterov) closed form
    a = ops["nest_a"] * 0.9 + ops["nest_g"]
    np.testing.assert_allclose(ops["nest_w1"], ops["nest_w"] - 3e-3 * ops["nest_g"] - 3e-3 * 0.9 * a, rtol=1e-6)
    np.testing.assert_array_equal(R.convert_image_dtype_u8(ops["u8"]), ops["u8_scaled"])
    assert ops["u8_scaled"][255] == np.float32(255) * np.float32(1 / 255)


def test_metrics_oracle_golden_and_sklearn():
    m = np.load(os.path.join(GOLDEN, "metrics.npz"))
    thr = list(m["thresholds"])
    tp, fp, fn, tn = MR.counts_at_thresholds(m["labels"], m["preds"], thr)
    for k, v in (("tp", tp), ("fp", fp), ("fn", fn), ("tn", tn)):
        np.testing.assert_array_equal(v, m[k])
    assert abs(MR.auc(m["labels"], m["preds"]) - float(m["auc"])) < 1e-7
    assert abs(MR.brier(m["labels"], m["preds"]) - float(m["brier"])) < 1e-12
    np.testing.assert_array_equal(MR.confusion_matrix(tp[-1], fp[-1], fn[-1], tn[-1]), m["confusion"])
    # the 200-threshold trapezoid approximates the exact ROC AUC
    sk = pytest.importorskip("sklearn.metrics")
    exact = sk.roc_auc_score(m["labels"].ravel(), m["preds"].ravel())
    assert abs(float(m["auc"]) - exact) < 5e-3
    # thresholds: [-eps, 1/199, ..., 198/199, 1-eps] (lib/metrics.py:4-8)
    assert thr[0] == -1e-7 and thr[199] == 1 - 1e-7 and abs(thr[1] - 1 / 199) < 1e-15 and thr[-1] == 0.5


def test_metric_known_answers():
    y = np.array([1, 1, 0, 0], np.float32)
    p = np.array([0.9, 0.4, 0.6, 0.1], np.float32)
    tp, fp, fn, tn = MR.counts_at_thresholds(y, p, [0.5])
    assert (tp[0], fp[0], fn[0], tn[0]) == (1, 1, 1, 1)
    # ties go to negative: pred == threshold is not positive (strict >)
    tp, fp, fn, tn = MR.counts_at_thresholds([1], [0.5], [0.5])
    assert (tp[0], fn[0]) == (0, 1)
    # perfect separation: AUC ~ 1
    assert MR.auc([0, 0, 1, 1], [0.1, 0.2, 0.8, 0.9]) > 0.99
    assert abs(MR.brier([1, 0], [0.5, 0.5]) - 0.25) < 1e-12
