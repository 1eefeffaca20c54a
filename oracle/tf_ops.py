"""numpy fp64 restatement of every TF op on the hot path (TEST ORACLE ONLY).

Parity unpinned (see oracle/__init__.py).  Each function names the reference
call site that instantiates the TF op and the TF semantics it restates
(SURVEY.md Appendix B).  Layouts: NHWC activations, HWIO kernels.
Written for clarity at small sizes, not speed.
"""
from __future__ import annotations

import numpy as np


# --------------------------------------------------------------- input scaling
def convert_image_dtype_u8(img_u8: np.ndarray) -> np.ndarray:
    """tf.image.convert_image_dtype(uint8 -> float32) at lib/dataset.py:20-21:
    cast to f32 then multiply by the f32 constant 1/255 (not x/255)."""
    return img_u8.astype(np.float32) * np.float32(1.0 / 255.0)


# ------------------------------------------------------------------- conv2d
def _pad_same(k: int) -> int:
    return (k - 1) // 2


def conv2d(x, w, stride=1, padding="same"):
    """TF Conv2D (NHWC, HWIO, no bias) as used by Keras conv2d_bn
    (train.py:129-130).  'same' at stride 1 pads (k-1)/2 on each side (every
    kernel here is odd); 'valid' pads nothing."""
    x = np.asarray(x, np.float64)
    w = np.asarray(w, np.float64)
    n, h, wd, ci = x.shape
    kh, kw, ci2, co = w.shape
    assert ci == ci2
    ph, pw = (_pad_same(kh), _pad_same(kw)) if padding == "same" else (0, 0)
    if padding == "same":
        assert stride == 1
    xp = np.pad(x, ((0, 0), (ph, ph), (pw, pw), (0, 0)))
    ho = (h + 2 * ph - kh) // stride + 1
    wo = (wd + 2 * pw - kw) // stride + 1
    y = np.zeros((n, ho, wo, co))
    for r in range(kh):
        for c in range(kw):
            patch = xp[:, r:r + stride * (ho - 1) + 1:stride, c:c + stride * (wo - 1) + 1:stride, :]
            y += patch @ w[r, c]
    return y


def conv2d_bwd_data(dy, w, x_shape, stride=1, padding="same"):
    """TF Conv2DBackpropInput (gradient of conv2d w.r.t. x)."""
    dy = np.asarray(dy, np.float64)
    w = np.asarray(w, np.float64)
    n, h, wd, ci = x_shape
    kh, kw, _, co = w.shape
    ph, pw = (_pad_same(kh), _pad_same(kw)) if padding == "same" else (0, 0)
    _, ho, wo, _ = dy.shape
    dxp = np.zeros((n, h + 2 * ph, wd + 2 * pw, ci))
    for r in range(kh):
        for c in range(kw):
            dxp[:, r:r + stride * (ho - 1) + 1:stride, c:c + stride * (wo - 1) + 1:stride, :] += dy @ w[r, c].T
    return dxp[:, ph:ph + h, pw:pw + wd, :]


def conv2d_bwd_filter(x, dy, w_shape, stride=1, padding="same"):
    """TF Conv2DBackpropFilter (gradient of conv2d w.r.t. the HWIO kernel)."""
    x = np.asarray(x, np.float64)
    dy = np.asarray(dy, np.float64)
    kh, kw, ci, co = w_shape
    ph, pw = (_pad_same(kh), _pad_same(kw)) if padding == "same" else (0, 0)
    xp = np.pad(x, ((0, 0), (ph, ph), (pw, pw), (0, 0)))
    _, ho, wo, _ = dy.shape
    dw = np.zeros(w_shape)
    for r in range(kh):
        for c in range(kw):
            patch = xp[:, r:r + stride * (ho - 1) + 1:stride, c:c + stride * (wo - 1) + 1:stride, :]
            dw[r, c] = patch.reshape(-1, ci).T @ dy.reshape(-1, co)
    return dw


# ------------------------------------------------------- batch norm + relu
def bn_relu_fwd(x, beta, eps=1e-3):
    """Keras BatchNormalization(scale=False) in training mode (always, App. C
    Q1: set_learning_phase(True) at train.py:101 before the model is built)
    followed by Activation('relu').  TF FusedBatchNorm: per-channel mean and
    BIASED variance over N*H*W; y = (x - mean) / sqrt(var + eps) + beta."""
    x = np.asarray(x, np.float64)
    axes = tuple(range(x.ndim - 1))
    mean = x.mean(axis=axes)
    var = ((x - mean) ** 2).mean(axis=axes)
    invstd = 1.0 / np.sqrt(var + eps)
    pre = (x - mean) * invstd + beta
    return np.maximum(pre, 0.0), mean, invstd


def bn_relu_bwd(dy, x, beta, eps=1e-3, mask=None):
    """ReluGrad (passes where the output is > 0) then FusedBatchNormGrad:
    dx = invstd * (g - mean(g) - xhat * mean(g * xhat)), dbeta = sum(g).
    `mask` (optional) overrides y > 0, so a checker can use the mask of the
    forward output under test (elements within an ulp of 0 may flip)."""
    x = np.asarray(x, np.float64)
    dy = np.asarray(dy, np.float64)
    axes = tuple(range(x.ndim - 1))
    y, mean, invstd = bn_relu_fwd(x, beta, eps)
    g = np.where(y > 0 if mask is None else mask, dy, 0.0)
    xhat = (x - mean) * invstd
    dbeta = g.sum(axis=axes)
    dx = invstd * (g - g.mean(axis=axes) - xhat * (g * xhat).mean(axis=axes))
    return dx, dbeta


# ------------------------------------------------------------------ pooling
def maxpool3x3s2(x):
    """MaxPooling2D((3,3), strides=(2,2)) 'valid' (InceptionV3 stem, mixed3,
    mixed8).  Returns y and the argmax window position (first max in scan
    order)."""
    x = np.asarray(x, np.float64)
    n, h, w, c = x.shape
    ho, wo = (h - 3) // 2 + 1, (w - 3) // 2 + 1
    taps = np.stack([x[:, r:r + 2 * (ho - 1) + 1:2, s:s + 2 * (wo - 1) + 1:2, :]
                     for r in range(3) for s in range(3)], axis=0)
    return taps.max(axis=0), taps.argmax(axis=0)


def maxpool3x3s2_bwd(dy, argmax, x_shape):
    """MaxPoolGrad: route each output gradient to its window's argmax."""
    n, h, w, c = x_shape
    _, ho, wo, _ = dy.shape
    dx = np.zeros(x_shape)
    for r in range(3):
        for s in range(3):
            m = (argmax == r * 3 + s)
            dx[:, r:r + 2 * (ho - 1) + 1:2, s:s + 2 * (wo - 1) + 1:2, :] += np.where(m, dy, 0.0)
    return dx


def _avg_counts(h, w):
    ch = np.array([1 + (i > 0) + (i < h - 1) for i in range(h)], np.float64)
    cw = np.array([1 + (j > 0) + (j < w - 1) for j in range(w)], np.float64)
    return ch[:, None] * cw[None, :]


def avgpool3x3s1_same(x):
    """AveragePooling2D((3,3), (1,1), 'same'): TF divides by the number of
    in-bounds taps (padding excluded from the count)."""
    x = np.asarray(x, np.float64)
    n, h, w, c = x.shape
    xp = np.pad(x, ((0, 0), (1, 1), (1, 1), (0, 0)))
    s = sum(xp[:, r:r + h, t:t + w, :] for r in range(3) for t in range(3))
    return s / _avg_counts(h, w)[None, :, :, None]


def avgpool3x3s1_same_bwd(dy):
    """AvgPoolGrad for the exclude-pad 3x3/1 'same' window."""
    dy = np.asarray(dy, np.float64)
    n, h, w, c = dy.shape
    g = dy / _avg_counts(h, w)[None, :, :, None]
    gp = np.pad(g, ((0, 0), (1, 1), (1, 1), (0, 0)))
    return sum(gp[:, r:r + h, t:t + w, :] for r in range(3) for t in range(3))


def global_avg_pool(x):
    """GlobalAveragePooling2D (pooling='avg', train.py:130)."""
    return np.asarray(x, np.float64).mean(axis=(1, 2))


# -------------------------------------------------------------------- head
def sigmoid(z):
    return 1.0 / (1.0 + np.exp(-np.asarray(z, np.float64)))


def dense(f, w, b):
    """tf.layers.dense(units=1) at train.py:133."""
    return np.asarray(f, np.float64) @ np.asarray(w, np.float64) + b


def sigmoid_xent_mean(z, y):
    """reduce_mean(sigmoid_cross_entropy_with_logits) at train.py:140-141:
    max(z,0) - z*y + log1p(exp(-|z|))."""
    z = np.asarray(z, np.float64)
    y = np.asarray(y, np.float64)
    return float(np.mean(np.maximum(z, 0) - z * y + np.log1p(np.exp(-np.abs(z)))))


def sigmoid_xent_grad(z, y):
    z = np.asarray(z, np.float64)
    return (sigmoid(z) - y) / z.size


# --------------------------------------------------------------- optimizers
def nesterov(w, g, a, lr=3e-3, m=0.9):
    """MomentumOptimizer(use_nesterov=True) at train.py:150-153 -> TF
    ApplyMomentum: accum = accum*m + g; var -= g*lr + accum*m*lr."""
    a = a * m + g
    w = w - (g * lr + a * m * lr)
    return w, a


def sgd(w, g, lr=3e-3):
    """GradientDescentOptimizer at train.py:147-148."""
    return w - lr * g


def momentum(w, g, a, lr=3e-3, m=0.9):
    """MomentumOptimizer(use_nesterov=False) (the -sgd-less, Nesterov-less
    form of train.py:150-153) -> TF ApplyMomentum: accum = accum*m + g;
    var -= accum*lr."""
    a = a * m + g
    return w - a * lr, a


def adam_beta_powers(t, b1=0.9, b2=0.999):
    """TF AdamOptimizer's fp32 beta1_power / beta2_power variables at step t
    (1-based): initialised to beta (fp32), multiplied by beta (fp32) after
    each step (optimizer._finish)."""
    f = np.float32
    p1, p2 = f(b1), f(b2)
    for _ in range(t - 1):
        p1, p2 = f(p1 * f(b1)), f(p2 * f(b2))
    return p1, p2


def adam_f32(w, g, m, v, t, lr=1e-3, b1=0.9, b2=0.999, eps=1e-8):
    """TF AdamOptimizer -> ApplyAdam (north-star extra; not used by the
    reference), restated in IEEE fp32 in TF's operation order (Eigen, no
    fused multiply-add): m += (g - m)(1 - b1); v += (g^2 - v)(1 - b2);
    var -= (m * alpha) / (sqrt(v) + eps), alpha = lr * sqrt(1 - beta2_power) /
    (1 - beta1_power) in fp32, left to right, from the fp32 beta-power
    variables (adam_beta_powers).  Returns (w, m, v, alpha) as float32."""
    f = np.float32
    w, g, m, v = (np.asarray(a, np.float32) for a in (w, g, m, v))
    p1, p2 = adam_beta_powers(t, b1, b2)
    alpha = f(f(f(lr) * np.sqrt(f(1) - p2)) / (f(1) - p1))
    one_b1, one_b2 = f(1) - f(b1), f(1) - f(b2)
    m = m + (g - m) * one_b1
    v = v + (g * g - v) * one_b2
    w = w - (m * alpha) / (np.sqrt(v) + f(eps))
    return w, m, v, alpha


def softmax_xent_mean(z, y):
    """Softmax-head mode (north-star extra): mean over samples of
    -sum_u y log softmax(z)_u; returns (loss, probs, dz)."""
    z = np.asarray(z, np.float64)
    y = np.asarray(y, np.float64)
    zm = z - z.max(axis=1, keepdims=True)
    p = np.exp(zm) / np.exp(zm).sum(axis=1, keepdims=True)
    lse = np.log(np.exp(zm).sum(axis=1, keepdims=True))
    loss = float(np.mean(np.sum(y * (lse - zm), axis=1)))
    return loss, p, (p - y) / z.shape[0]
