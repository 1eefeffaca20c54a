"""Checkpoints in place of tf.train.Saver (train.py:207,267,273-274;
evaluate.py:174-175).

A checkpoint at `path` is three files, so the ensemble glob of
evaluate.py:78-85 (".".join(name.split(".")[:-1]) over glob(path*), deduped)
recovers `path` exactly as it does for TF's `.meta/.index/.data-*` trio:
  <path>.meta                   JSON: graph config (resolution, units, op
                                order) and the parameter table
  <path>.index                  JSON: name -> (shape, offset, size), sha256
  <path>.data-00000-of-00001    raw little-endian float32, the flat
                                parameter buffer (jr.init.param_layout)
Loading executes nothing from the files (JSON + raw floats only).
"""
from __future__ import annotations

import hashlib
import json
import os
from typing import Tuple

import numpy as np

from .init import param_layout

DATA_SUFFIX = ".data-00000-of-00001"
FORMAT = "jr-checkpoint-v1"


def save(path: str, graph, flat: np.ndarray, extra: dict | None = None) -> None:
    layout, total = param_layout(graph.params)
    flat = np.ascontiguousarray(flat, dtype="<f4")
    if flat.size != total:
        raise ValueError(f"flat parameter vector has {flat.size} values, layout needs {total}")
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    raw = flat.tobytes()
    meta = {"format": FORMAT, "height": graph.height, "width": graph.width, "units": graph.units,
            "model": "inception_v3", "num_params": graph.num_params(), **(extra or {})}
    index = {"format": FORMAT, "total": total, "sha256": hashlib.sha256(raw).hexdigest(),
             "tensors": [{"name": n, "shape": list(s), "offset": o, "size": z} for n, s, o, z in layout]}
    tmp = path + DATA_SUFFIX + ".tmp"
    with open(tmp, "wb") as f:
        f.write(raw)
    os.replace(tmp, path + DATA_SUFFIX)
    with open(path + ".index", "w") as f:
        json.dump(index, f)
    with open(path + ".meta", "w") as f:
        json.dump(meta, f, indent=1)


def load(path: str, graph=None, verify: bool = True) -> Tuple[np.ndarray, dict]:
    """(flat float32 parameters, meta dict).  With `graph`, the tensor table
    must match its parameter layout exactly."""
    with open(path + ".meta") as f:
        meta = json.load(f)
    with open(path + ".index") as f:
        index = json.load(f)
    if meta.get("format") != FORMAT or index.get("format") != FORMAT:
        raise ValueError(f"{path}: not a {FORMAT} checkpoint")
    raw = open(path + DATA_SUFFIX, "rb").read()
    if verify and hashlib.sha256(raw).hexdigest() != index["sha256"]:
        raise ValueError(f"{path}: data checksum mismatch")
    flat = np.frombuffer(raw, dtype="<f4").astype(np.float32)
    if flat.size != index["total"]:
        raise ValueError(f"{path}: data size mismatch")
    if graph is not None:
        layout, total = param_layout(graph.params)
        want = [(n, list(s), o, z) for n, s, o, z in layout]
        got = [(t["name"], t["shape"], t["offset"], t["size"]) for t in index["tensors"]]
        if want != got or total != index["total"]:
            raise ValueError(f"{path}: parameter table does not match the model graph")
    return flat, meta


def read_meta(path: str) -> dict:
    """The graph configuration of a checkpoint, from <path>.meta only (no
    parameter read or checksum): what evaluate.py needs to size its engines."""
    with open(path + ".meta") as f:
        meta = json.load(f)
    if meta.get("format") != FORMAT:
        raise ValueError(f"{path}: not a {FORMAT} checkpoint")
    return meta


def exists(path: str) -> bool:
    return all(os.path.exists(path + s) for s in (".meta", ".index", DATA_SUFFIX))
