"""Seeded parameter initialisation (Keras defaults).

The reference loads ImageNet weights at train.py:129-130 but then re-runs
every initializer with `sess.run(tf.global_variables_initializer())` at
train.py:210, so training starts from the Keras
default initializers [TF-3P]:
  Conv2D kernel   glorot_uniform  limit = sqrt(6 / (fan_in + fan_out)),
                  fan_in = kh*kw*cin, fan_out = kh*kw*cout
  BN beta         zeros
  Dense kernel    glorot_uniform  fan_in = 2048, fan_out = units
  Dense bias      zeros
The stream of draws (numpy PCG64(seed), parameters in Keras creation order)
is ours: TF's own RNG stream is not reproducible outside TF.  Ensemble member
m uses seed m.
"""
from __future__ import annotations

import numpy as np

ALIGN = 64  # floats; every parameter tensor starts on a 256-byte boundary


def param_layout(params):
    """[(name, shape, offset, size)] in the flat buffer, and the padded total."""
    out = []
    off = 0
    for name, shape in params:
        size = int(np.prod(shape))
        out.append((name, tuple(shape), off, size))
        off += (size + ALIGN - 1) // ALIGN * ALIGN
    return out, off


def glorot_limit(shape) -> float:
    if len(shape) == 4:
        rf = shape[0] * shape[1]
        fan_in, fan_out = rf * shape[2], rf * shape[3]
    else:
        fan_in, fan_out = shape[0], shape[1]
    return float(np.sqrt(6.0 / (fan_in + fan_out)))


def init_params(graph, seed: int = 0) -> np.ndarray:
    """Flat float32 parameter vector (padding = 0) for `graph` (jr.inception)."""
    layout, total = param_layout(graph.params)
    flat = np.zeros(total, dtype=np.float32)
    rng = np.random.Generator(np.random.PCG64(seed))
    for name, shape, off, size in layout:
        if name.endswith("/kernel"):
            lim = glorot_limit(shape)
            flat[off:off + size] = rng.uniform(-lim, lim, size=size).astype(np.float32)
        # betas and biases stay zero
    return flat


def unflatten(graph, flat: np.ndarray) -> dict:
    layout, _ = param_layout(graph.params)
    return {name: flat[off:off + size].reshape(shape) for name, shape, off, size in layout}
