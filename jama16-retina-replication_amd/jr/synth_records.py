"""Write synthetic fundus TFRecords in the create_tfrecords schema that
lib/dataset.py:12-16 parses (image/encoded JPEG q=100 as lib/preprocess.py
:173-174 writes it, image/format, image/class/label, image/height,
image/width), sharded like eyepacs.sh:224-234 (--num_shards)."""
from __future__ import annotations

import io
import os

import numpy as np
from PIL import Image

from . import synth, tfrecord


def encode_jpeg(img: np.ndarray, quality: int = 100) -> bytes:
    buf = io.BytesIO()
    Image.fromarray(img).save(buf, format="JPEG", quality=quality)
    return buf.getvalue()


def write_split(out_dir: str, n: int, size: int = 299, p: float = synth.P_TRAIN, start: int = 0,
                num_shards: int = 2, name: str = "train", label_seed: int = 7) -> None:
    os.makedirs(out_dir, exist_ok=True)
    labels = synth.labels(start, n, p, seed=label_seed)
    per = (n + num_shards - 1) // num_shards
    for s in range(num_shards):
        path = os.path.join(out_dir, f"{name}-{s:05d}-of-{num_shards:05d}.tfrecord")
        with tfrecord.TFRecordWriter(path) as w:
            for i in range(s * per, min(n, (s + 1) * per)):
                img = synth.fundus_image(start + i, size)
                w.write(tfrecord.encode_example({
                    "image/encoded": encode_jpeg(img),
                    "image/format": b"jpeg",
                    "image/class/label": int(labels[i, 0]),
                    "image/height": size,
                    "image/width": size,
                }))
