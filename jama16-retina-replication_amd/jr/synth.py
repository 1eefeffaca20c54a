"""Synthetic fundus-shaped images and labels.

No real EyePACS / Messidor data is available (no network).  Images mimic what
lib/preprocess.py:79-130,173-174 produces: a black square with a centred
retina disc whose diameter equals the side, orange-red base colour
(~(180, 85, 40) with per-image jitter), Gaussian noise sigma 8, and a few dark
vessel-like strokes.  Image i uses numpy PCG64(432 + i) (432 = the
reference's random.seed, train.py:17).  Labels are Bernoulli with the
EyePACS bin2 prevalence: 0.288 train (16458/57146, eyepacs.sh:176-177),
0.079 test (696/8792).
"""
from __future__ import annotations

import numpy as np

P_TRAIN = 16458 / 57146
P_TEST = 696 / 8792


def fundus_image(i: int, size: int = 299) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(432 + i))
    yy, xx = np.mgrid[0:size, 0:size].astype(np.float32)
    c = (size - 1) / 2.0
    r = np.sqrt((yy - c) ** 2 + (xx - c) ** 2)
    disc = r <= size / 2.0
    base = np.array([180.0, 85.0, 40.0], np.float32) + rng.normal(0, 12, 3).astype(np.float32)
    # radial vignetting + optic-disc bright spot
    shade = (1.0 - 0.35 * (r / (size / 2.0)) ** 2)[..., None]
    od_y, od_x = c + rng.uniform(-0.1, 0.1) * size, c + rng.uniform(0.15, 0.3) * size * rng.choice([-1, 1])
    od = np.exp(-((yy - od_y) ** 2 + (xx - od_x) ** 2) / (2 * (0.06 * size) ** 2))[..., None]
    img = base * shade + od * np.array([60.0, 60.0, 40.0], np.float32)
    # vessels: a few dark sinusoidal strokes radiating from the optic disc
    for _ in range(int(rng.integers(4, 9))):
        ang = rng.uniform(0, 2 * np.pi)
        amp, freq, ph = rng.uniform(2, 10), rng.uniform(0.01, 0.04), rng.uniform(0, 2 * np.pi)
        dx, dy = np.cos(ang), np.sin(ang)
        t = (xx - od_x) * dx + (yy - od_y) * dy
        perp = -(xx - od_x) * dy + (yy - od_y) * dx - amp * np.sin(freq * t + ph)
        width = rng.uniform(1.0, 3.0) * size / 299.0
        mask = (np.abs(perp) < width) & (t > 0)
        img = np.where(mask[..., None], img * 0.55, img)
    img = img + rng.normal(0, 8.0, img.shape).astype(np.float32)
    img = np.where(disc[..., None], img, 0.0)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def fundus_batch(start: int, n: int, size: int = 299) -> np.ndarray:
    return np.stack([fundus_image(start + k, size) for k in range(n)])


def labels(start: int, n: int, p: float = P_TRAIN, seed: int = 7) -> np.ndarray:
    """Bernoulli(p) labels, deterministic per index."""
    out = np.empty((n, 1), np.float32)
    for k in range(n):
        rng = np.random.Generator(np.random.PCG64(seed * 1_000_003 + start + k))
        out[k, 0] = 1.0 if rng.random() < p else 0.0
    return out
