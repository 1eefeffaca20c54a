"""Minimal TensorBoard event writer (tf.summary.FileWriter + scalar summary,
train.py:181,187-189, lib/evaluation.py:71-72) without TF.

Event files are TFRecord containers of `Event` protos:
  Event{1: wall_time (double), 2: step (int64), 3: file_version (string),
        5: summary Summary{1: repeated Value{1: tag (string),
        2: simple_value (float)}}}
"""
from __future__ import annotations

import os
import socket
import struct
import time

from . import tfrecord


def _event(wall: float, step: int, *, file_version: str | None = None, scalars: dict | None = None) -> bytes:
    out = tfrecord._field(1, 1, struct.pack("<d", wall))
    out += tfrecord._varint((2 << 3) | 0) + tfrecord._varint(int(step))
    if file_version is not None:
        out += tfrecord._field(3, 2, file_version.encode())
    if scalars:
        summ = b""
        for tag, v in scalars.items():
            val = tfrecord._field(1, 2, tag.encode()) + tfrecord._field(2, 5, struct.pack("<f", float(v)))
            summ += tfrecord._field(1, 2, val)
        out += tfrecord._field(5, 2, summ)
    return out


class FileWriter:
    def __init__(self, logdir: str):
        os.makedirs(logdir, exist_ok=True)
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}"
        self.path = os.path.join(logdir, name)
        self._w = tfrecord.TFRecordWriter(self.path)
        self._w.write(_event(time.time(), 0, file_version="brain.Event:2"))
        self._w._f.flush()

    def add_scalars(self, scalars: dict, step: int) -> None:
        self._w.write(_event(time.time(), step, scalars=scalars))
        self._w._f.flush()

    def add_summary(self, summary: dict, step) -> None:
        """train.py's summary_writer.add_summary(summaries, epoch)."""
        self.add_scalars(summary, 0 if step is None else step)

    def close(self) -> None:
        self._w.close()
