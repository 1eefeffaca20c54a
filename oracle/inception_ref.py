"""torch-CPU restatement of the reference training step (TEST ORACLE ONLY).

Parity unpinned (oracle/__init__.py).  Restates, independently of the product
graph builder, the graph the reference builds at train.py:128-153:
  InceptionV3(include_top=False, pooling='avg') [TF-3P keras_applications
  inception_v3.py, written out below in its own conv2d_bn style],
  dense(units=1) (train.py:133), sigmoid 'predictions' (train.py:136),
  reduce_mean(sigmoid_cross_entropy_with_logits) (train.py:140-141),
  MomentumOptimizer(3e-3, 0.9, use_nesterov=True) or GradientDescent
  (train.py:146-153), with BN always in batch-statistics mode (App. C Q1).
Backward is torch autograd.  Runs in fp64 for goldens and fp32 for the
CPU baseline timing in bench.py (kind "port").

emulate_bf16=True is an independent bf16 implementation of the same step
for the bf16 envelope of tests/test_gpu_baseline_sizes.py: it rounds to bf16
(RNE) where the bf16 GPU path stores bf16 -- the input image, every filter,
every raw conv output (BN statistics then see the stored values), every BN+ReLU
output and average-pool output -- and, in the backward, the gradients of those
stored tensors (custom autograd rounding both ways); arithmetic stays in the
oracle's dtype (fp64).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

EPS = 1e-3


class _RoundBF16(torch.autograd.Function):
    """bf16 storage: round the value forward and its gradient backward."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


class InceptionV3Ref:
    """Functional Inception-v3 over a {name: tensor} parameter dict (HWIO)."""

    def __init__(self, params: dict, dtype=torch.float64, requires_grad=True, emulate_bf16=False,
                 order_seed=None):
        self.dtype = dtype
        self.bf16 = emulate_bf16
        # order_seed: the same arithmetic with every reduction in another fp32
        # order -- each conv's input channels permuted (its Cin sum and the
        # data-gradient's channel order), the images of each batch permuted
        # (BN statistics, filter gradients, the loss mean).  Exact in real
        # arithmetic; an independent fp32 sample of the loss curve for the
        # calibration of the fp32 curve bar (oracle/make_golden.py curvecal)
        self.order = np.random.default_rng(order_seed) if order_seed is not None else None
        self.P = {k: torch.tensor(np.asarray(v), dtype=dtype, requires_grad=requires_grad)
                  for k, v in params.items()}
        self._k = 0
        self.record = None   # set to [] to keep every conv2d_bn output (and its grad)

    # keras_applications.inception_v3.conv2d_bn
    def conv2d_bn(self, x, filters, num_row, num_col, padding="same", strides=(1, 1)):
        self._k += 1
        w = self.P[f"conv2d_{self._k}/kernel"]
        beta = self.P[f"batch_normalization_{self._k}/beta"]
        assert tuple(w.shape) == (num_row, num_col, x.shape[1], filters), (self._k, tuple(w.shape))
        pad = ((num_row - 1) // 2, (num_col - 1) // 2) if padding == "same" else (0, 0)
        if self.order is not None:
            perm = torch.as_tensor(self.order.permutation(x.shape[1]))
            x, w = x[:, perm], w[:, :, perm, :]
        y = F.conv2d(x, self._r(w).permute(3, 2, 0, 1), stride=strides, padding=pad)
        y = self._r(y)                                                  # raw output as stored
        mean = y.mean(dim=(0, 2, 3), keepdim=True)
        var = ((y - mean) ** 2).mean(dim=(0, 2, 3), keepdim=True)      # biased
        y = (y - mean) / torch.sqrt(var + EPS) + beta.view(1, -1, 1, 1)
        y = self._r(F.relu(y))
        if self.record is not None:          # debugging aid: keep every block output
            if y.requires_grad:
                y.retain_grad()
            self.record.append(y)
        return y

    def _r(self, t):
        return _RoundBF16.apply(t) if self.bf16 else t

    @staticmethod
    def maxpool(x):
        return F.max_pool2d(x, 3, 2)

    def avgpool_same(self, x):
        return self._r(F.avg_pool2d(x, 3, 1, padding=1, count_include_pad=False))

    def features(self, x_nhwc):
        self._k = 0
        cb = self.conv2d_bn
        x = self._r(x_nhwc.permute(0, 3, 1, 2))
        x = cb(x, 32, 3, 3, strides=(2, 2), padding="valid")
        x = cb(x, 32, 3, 3, padding="valid")
        x = cb(x, 64, 3, 3)
        x = self.maxpool(x)
        x = cb(x, 80, 1, 1, padding="valid")
        x = cb(x, 192, 3, 3, padding="valid")
        x = self.maxpool(x)
        for pool_f in (32, 64, 64):                      # mixed 0, 1, 2
            b1 = cb(x, 64, 1, 1)
            b5 = cb(cb(x, 48, 1, 1), 64, 5, 5)
            b3 = cb(cb(cb(x, 64, 1, 1), 96, 3, 3), 96, 3, 3)
            bp = cb(self.avgpool_same(x), pool_f, 1, 1)
            x = torch.cat([b1, b5, b3, bp], 1)
        b3 = cb(x, 384, 3, 3, strides=(2, 2), padding="valid")   # mixed 3
        bd = cb(cb(cb(x, 64, 1, 1), 96, 3, 3), 96, 3, 3, strides=(2, 2), padding="valid")
        x = torch.cat([b3, bd, self.maxpool(x)], 1)
        for c7 in (128, 160, 160, 192):                  # mixed 4..7
            b1 = cb(x, 192, 1, 1)
            b7 = cb(cb(cb(x, c7, 1, 1), c7, 1, 7), 192, 7, 1)
            bd = cb(x, c7, 1, 1)
            bd = cb(bd, c7, 7, 1)
            bd = cb(bd, c7, 1, 7)
            bd = cb(bd, c7, 7, 1)
            bd = cb(bd, 192, 1, 7)
            bp = cb(self.avgpool_same(x), 192, 1, 1)
            x = torch.cat([b1, b7, bd, bp], 1)
        b3 = cb(cb(x, 192, 1, 1), 320, 3, 3, strides=(2, 2), padding="valid")   # mixed 8
        b7 = cb(cb(cb(cb(x, 192, 1, 1), 192, 1, 7), 192, 7, 1), 192, 3, 3, strides=(2, 2),
                padding="valid")
        x = torch.cat([b3, b7, self.maxpool(x)], 1)
        for _ in range(2):                                # mixed 9, 10
            b1 = cb(x, 320, 1, 1)
            b3 = cb(x, 384, 1, 1)
            b3 = torch.cat([cb(b3, 384, 1, 3), cb(b3, 384, 3, 1)], 1)
            bd = cb(cb(x, 448, 1, 1), 384, 3, 3)
            bd = torch.cat([cb(bd, 384, 1, 3), cb(bd, 384, 3, 1)], 1)
            bp = cb(self.avgpool_same(x), 192, 1, 1)
            x = torch.cat([b1, b3, bd, bp], 1)
        assert self._k == 94
        return x.mean(dim=(2, 3))                         # GlobalAveragePooling2D

    def forward(self, x_nhwc, labels=None):
        x = torch.as_tensor(np.asarray(x_nhwc), dtype=self.dtype)
        f = self.features(x)
        logits = f @ self.P["dense/kernel"] + self.P["dense/bias"]
        probs = torch.sigmoid(logits)
        loss = None
        if labels is not None:
            y = torch.as_tensor(np.asarray(labels), dtype=self.dtype).reshape(logits.shape)
            loss = torch.mean(torch.clamp(logits, min=0) - logits * y + torch.log1p(torch.exp(-logits.abs())))
        return logits, probs, loss

    def train_step(self, x_nhwc, labels, state: dict, lr=3e-3, momentum=0.9, nesterov=True, sgd=False):
        """One reference step: forward, loss, gradients, ApplyMomentum/SGD.
        Returns (loss, probs, grads{name: ndarray})."""
        for p in self.P.values():
            p.grad = None
        if self.order is not None:
            bp = self.order.permutation(len(x_nhwc))
            x_nhwc = np.asarray(x_nhwc)[bp]
            labels = np.asarray(labels).reshape(len(bp), -1)[bp]
        logits, probs, loss = self.forward(x_nhwc, labels)
        self.last_logits = logits.detach().cpu().numpy().copy()
        loss.backward()
        grads = {}
        with torch.no_grad():
            for k, p in self.P.items():
                g = p.grad if p.grad is not None else torch.zeros_like(p)
                grads[k] = g.detach().cpu().numpy().copy()
                if sgd:
                    p -= lr * g
                else:
                    a = state.setdefault(k, torch.zeros_like(p))
                    a.mul_(momentum).add_(g)
                    if nesterov:
                        p -= g * lr + a * momentum * lr
                    else:
                        p -= a * lr
        return float(loss.item()), probs.detach().cpu().numpy(), grads

    def params_numpy(self) -> dict:
        return {k: v.detach().cpu().numpy().copy() for k, v in self.P.items()}
