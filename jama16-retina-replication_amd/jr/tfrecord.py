"""TFRecord container + tf.train.Example codec, without TensorFlow.

The reference reads `*.tfrecord` files with tf.data.TFRecordDataset
(lib/dataset.py:5-8) and parses each record with parse_single_example over
five features (lib/dataset.py:12-17):
  image/encoded (bytes, JPEG), image/format (bytes), image/class/label
  (int64), image/height (int64), image/width (int64)
as written by the (non-vendored) create_tfrecords submodule
(eyepacs.sh:224-234).  This module restates the two wire formats [TF-3P]:

TFRecord:  uint64le length | uint32le masked_crc32c(length bytes) | data |
           uint32le masked_crc32c(data)       (CRC32C from libjr, SSE4.2)
Example:   protobuf  Example{1: Features{1: map<string, Feature>}}
           Feature{1: BytesList{1: repeated bytes} | 2: FloatList{1: packed
           float} | 3: Int64List{1: packed int64}}
"""
from __future__ import annotations

import ctypes
import mmap
import os
import struct
from typing import Dict, Iterator, List, Union

import numpy as np

from . import _ffi

FeatureValue = Union[bytes, int, float, List[bytes], List[int], List[float], np.ndarray]


def _check_host(name: str, rc: int) -> None:
    if rc != _ffi.JR_OK:
        raise _ffi.JRError(name, rc, _ffi.host_last_error())


# ------------------------------------------------------------------ CRC32C
def _ptr(data) -> bytes:
    # a bytes object is passed to the C-ABI as a pointer to its own buffer
    # (no copy: the record payloads are ~80 KB JPEGs, read once per record)
    return data if isinstance(data, bytes) else bytes(data)


def masked_crc32c(data: bytes) -> int:
    lib = _ffi.load_host()
    b = _ptr(data)
    return int(lib.jr_masked_crc32c(b, len(b)))


def crc32c(data: bytes, crc: int = 0) -> int:
    lib = _ffi.load_host()
    b = _ptr(data)
    return int(lib.jr_crc32c(b, len(b), crc))


# --------------------------------------------------------------- container
class TFRecordError(IOError):
    pass


def read_records(path: str, verify: bool = True) -> Iterator[bytes]:
    """Yield the payload of every record of one TFRecord file, in order."""
    with open(path, "rb") as f:
        while True:
            head = f.read(12)
            if not head:
                return
            if len(head) < 12:
                raise TFRecordError(f"{path}: truncated record header")
            (length,) = struct.unpack("<Q", head[:8])
            (len_crc,) = struct.unpack("<I", head[8:12])
            if verify and masked_crc32c(head[:8]) != len_crc:
                raise TFRecordError(f"{path}: corrupted record length")
            data = f.read(length)
            tail = f.read(4)
            if len(data) < length or len(tail) < 4:
                raise TFRecordError(f"{path}: truncated record")
            if verify and masked_crc32c(data) != struct.unpack("<I", tail)[0]:
                raise TFRecordError(f"{path}: corrupted record data")
            yield data


_KEYS = ("image/encoded", "image/format", "image/class/label", "image/height", "image/width")


class RecordFile:
    """One TFRecord file, mmap'd and indexed by libjr (jr_tfrecord_index), with
    the lib/dataset.py:12-16 features of every record located natively
    (jr_example_parse_image).  Records past a damaged one are not indexed;
    `raise_if_damaged()` raises the TFRecordError the Python reader would have
    raised on reaching it."""

    def __init__(self, path: str, verify: bool = True, parse: bool = True):
        lib = _ffi.load_host()
        self.path = path
        size = os.path.getsize(path)
        self._mm = None
        if size:
            with open(path, "rb") as fh:
                self._mm = mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_READ)
            self.buf = np.frombuffer(self._mm, np.uint8)
        else:
            self.buf = np.zeros(1, np.uint8)
        base = self.buf.ctypes.data
        n = ctypes.c_size_t(0)
        rc = lib.jr_tfrecord_index(base, size, int(verify), None, None, 0, ctypes.byref(n))
        self.error = None if rc == 0 else _ffi.host_last_error()
        cnt = n.value
        self.offsets = np.zeros(cnt, np.uint64)
        self.lengths = np.zeros(cnt, np.uint64)
        if cnt:
            rc2 = lib.jr_tfrecord_index(base, size, int(verify), self.offsets.ctypes.data,
                                        self.lengths.ctypes.data, cnt, ctypes.byref(n))
            if rc2 != rc or n.value != cnt:       # the damage (if any) is where the count stopped
                raise TFRecordError(f"{path}: changed while being indexed")
        self.num_records = cnt
        if parse:
            self.enc_off = np.zeros(cnt, np.uint64)
            self.enc_len = np.zeros(cnt, np.uint64)
            self.label = np.zeros(cnt, np.int64)
            self.height = np.zeros(cnt, np.int64)
            self.width = np.zeros(cnt, np.int64)
            self.status = np.zeros(cnt, np.int32)
            _check_host("jr_example_parse_image", lib.jr_example_parse_image(
                base, self.offsets.ctypes.data, self.lengths.ctypes.data, cnt, self.enc_off.ctypes.data,
                self.enc_len.ctypes.data, self.label.ctypes.data, self.height.ctypes.data,
                self.width.ctypes.data, self.status.ctypes.data))

    def record(self, i: int) -> bytes:
        o = int(self.offsets[i])
        return self.buf[o:o + int(self.lengths[i])].tobytes()

    def check(self, i: int) -> None:
        st = int(self.status[i])
        if st < 0:
            raise ValueError(f"{self.path}: record {i} is not a serialized tf.train.Example")
        if st:
            key = _KEYS[(st & -st).bit_length() - 1]
            raise ValueError(f"record is missing FixedLenFeature {key!r}")

    def encoded(self, i: int) -> memoryview:
        """The image/encoded bytes of record i (a view into the mapping)."""
        o = int(self.enc_off[i])
        return memoryview(self.buf[o:o + int(self.enc_len[i])])

    def raise_if_damaged(self) -> None:
        if self.error is not None:
            raise TFRecordError(f"{self.path}: {self.error}")


class TFRecordWriter:
    def __init__(self, path: str):
        self._f = open(path, "wb")

    def write(self, data: bytes) -> None:
        length = struct.pack("<Q", len(data))
        self._f.write(length)
        self._f.write(struct.pack("<I", masked_crc32c(length)))
        self._f.write(data)
        self._f.write(struct.pack("<I", masked_crc32c(data)))

    def close(self) -> None:
        self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


# ---------------------------------------------------------------- protobuf
def _varint(v: int) -> bytes:
    if v < 0:
        v += 1 << 64
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf: bytes, pos: int):
    shift = 0
    result = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7
        if shift > 63:
            raise ValueError("varint too long")


def _field(num: int, wire: int, payload: bytes) -> bytes:
    key = _varint((num << 3) | wire)
    if wire == 2:
        return key + _varint(len(payload)) + payload
    return key + payload


def _feature(value: FeatureValue) -> bytes:
    if isinstance(value, (bytes, bytearray)):
        value = [bytes(value)]
    if isinstance(value, (int, np.integer)):
        value = [int(value)]
    if isinstance(value, (float, np.floating)):
        value = [float(value)]
    value = list(value)
    if all(isinstance(v, (bytes, bytearray)) for v in value):
        inner = b"".join(_field(1, 2, bytes(v)) for v in value)
        return _field(1, 2, inner)                      # bytes_list
    if all(isinstance(v, (int, np.integer)) for v in value):
        packed = b"".join(_varint(int(v)) for v in value)
        return _field(3, 2, _field(1, 2, packed))       # int64_list (packed)
    packed = struct.pack(f"<{len(value)}f", *[float(v) for v in value])
    return _field(2, 2, _field(1, 2, packed))           # float_list (packed)


def encode_example(features: Dict[str, FeatureValue]) -> bytes:
    entries = b""
    for key in sorted(features):
        entry = _field(1, 2, key.encode()) + _field(2, 2, _feature(features[key]))
        entries += _field(1, 2, entry)
    return _field(1, 2, entries)


def _parse_list(buf: bytes, kind: int):
    """Decode BytesList(1) / FloatList(2) / Int64List(3) payloads."""
    pos, out = 0, []
    while pos < len(buf):
        key, pos = _read_varint(buf, pos)
        num, wire = key >> 3, key & 7
        if num != 1:
            raise ValueError("unexpected field in feature list")
        if kind == 1:
            n, pos = _read_varint(buf, pos)
            out.append(bytes(buf[pos:pos + n]))
            pos += n
        elif kind == 2:
            if wire == 2:
                n, pos = _read_varint(buf, pos)
                out.extend(struct.unpack(f"<{n // 4}f", buf[pos:pos + n]))
                pos += n
            else:
                out.append(struct.unpack("<f", buf[pos:pos + 4])[0])
                pos += 4
        else:
            if wire == 2:
                n, pos = _read_varint(buf, pos)
                end = pos + n
                while pos < end:
                    v, pos = _read_varint(buf, pos)
                    out.append(v - (1 << 64) if v >= 1 << 63 else v)
            else:
                v, pos = _read_varint(buf, pos)
                out.append(v - (1 << 64) if v >= 1 << 63 else v)
    return out


def _skip(buf: bytes, pos: int, wire: int) -> int:
    if wire == 0:
        _, pos = _read_varint(buf, pos)
        return pos
    if wire == 1:
        return pos + 8
    if wire == 2:
        n, pos = _read_varint(buf, pos)
        return pos + n
    if wire == 5:
        return pos + 4
    raise ValueError(f"unsupported wire type {wire}")


def decode_example(data: bytes) -> Dict[str, list]:
    """tf.train.Example bytes -> {feature name: list of values}."""
    out: Dict[str, list] = {}
    pos = 0
    while pos < len(data):
        key, pos = _read_varint(data, pos)
        if key >> 3 != 1 or key & 7 != 2:
            pos = _skip(data, pos, key & 7)
            continue
        n, pos = _read_varint(data, pos)
        feats, pos = data[pos:pos + n], pos + n
        fpos = 0
        while fpos < len(feats):
            k2, fpos = _read_varint(feats, fpos)
            if k2 >> 3 != 1 or k2 & 7 != 2:
                fpos = _skip(feats, fpos, k2 & 7)
                continue
            n2, fpos = _read_varint(feats, fpos)
            entry, fpos = feats[fpos:fpos + n2], fpos + n2
            epos, name, value = 0, None, []
            while epos < len(entry):
                k3, epos = _read_varint(entry, epos)
                n3, epos = _read_varint(entry, epos)
                payload, epos = entry[epos:epos + n3], epos + n3
                if k3 >> 3 == 1:
                    name = payload.decode()
                elif k3 >> 3 == 2:
                    fp = 0
                    while fp < len(payload):
                        k4, fp = _read_varint(payload, fp)
                        n4, fp = _read_varint(payload, fp)
                        value = _parse_list(payload[fp:fp + n4], k4 >> 3)
                        fp += n4
            if name is not None:
                out[name] = value
    return out
