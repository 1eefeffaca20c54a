"""Native JPEG decode (libjr_jpeg.so, include/jr_jpeg.h) for lib/dataset.py.

tf.image.decode_jpeg (lib/dataset.py:20) decodes with libjpeg-turbo's IFAST
IDCT by default [TF-3P]; this decoder runs IJG libjpeg 9 with the IDCT
selectable ("ifast" = TF's default, "islow" = Pillow's), entirely outside
the interpreter, so the pipeline's worker threads decode in parallel.  It is
optional host plumbing: when libjr_jpeg.so is absent the pipeline decodes
with Pillow (ISLOW).  Chroma upsampling of 4:2:0 files differs between IJG 9
and libjpeg-turbo by a few LSB (decode parity unpinned).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("JR_JPEG_LIB", os.path.join(_HERE, "libjr_jpeg.so"))
DCT = {"ifast": 0, "islow": 1}
_lib = None


def load() -> Optional[ctypes.CDLL]:
    """The decoder library, or None when it is not built."""
    global _lib
    if _lib is not None:
        return _lib or None
    if not os.path.exists(LIB_PATH):
        _lib = False
        return None
    lib = ctypes.CDLL(LIB_PATH)
    lib.jr_jpeg_last_error.restype = ctypes.c_char_p
    lib.jr_jpeg_header.restype = ctypes.c_int
    lib.jr_jpeg_header.argtypes = [ctypes.c_void_p, ctypes.c_size_t] + [ctypes.POINTER(ctypes.c_int32)] * 3
    lib.jr_jpeg_decode.restype = ctypes.c_int
    lib.jr_jpeg_decode.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int32,
                                   ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]
    _lib = lib
    return lib


def available() -> bool:
    return load() is not None


def _buf(data):
    """(pointer, length, keep-alive) of any bytes-like object (bytes, a
    memoryview into a mapped TFRecord file, ...), without a copy."""
    a = np.frombuffer(data, np.uint8)
    return a.ctypes.data, a.size, a


def header(data):
    lib = load()
    p, n, _keep = _buf(data)
    h, w, c = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    if lib.jr_jpeg_header(p, n, ctypes.byref(h), ctypes.byref(w), ctypes.byref(c)) != 0:
        raise ValueError(f"JPEG header: {lib.jr_jpeg_last_error().decode(errors='replace')}")
    return h.value, w.value, c.value


def decode(data, dct: str = "ifast", out: Optional[np.ndarray] = None) -> np.ndarray:
    """HWC uint8 with the file's channels (tf.image.decode_jpeg channels=0);
    into `out` (a C-contiguous uint8 array of exactly that size) if given."""
    lib = load()
    if lib is None:
        raise RuntimeError("libjr_jpeg.so is not built")
    h, w, c = header(data)
    if out is None:
        out = np.empty((h, w, c), np.uint8)
    elif out.dtype != np.uint8 or out.size != h * w * c or not out.flags.c_contiguous:
        raise ValueError(f"cannot decode a {h}x{w}x{c} image into a buffer of {out.size} uint8")
    p, n, _keep = _buf(data)
    if lib.jr_jpeg_decode(p, n, out.ctypes.data, h, w, c, DCT[dct]) != 0:
        raise ValueError(f"JPEG decode: {lib.jr_jpeg_last_error().decode(errors='replace')}")
    return out
