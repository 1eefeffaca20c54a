"""Data-parallel gradient exchange: bucketed all-reduce overlapped with backward.

The reference's only multi-GPU path is an external tf_cnn_benchmarks
parameter server (benchmarks.yaml.jinja.example:81-90; SURVEY.md §2 row 14,
§8e).  Here every rank keeps a full replica, computes BN statistics on its
own 64 images (the reference's per-batch-of-64 semantics), and the flat fp32
gradient (87.1 MB) is summed with torch.distributed all_reduce — backend
'nccl' is RCCL over xGMI on MI355X ('gloo' on CPU for tests).

Buckets are contiguous ranges of the flat gradient, cut at parameter-tensor
boundaries, issued in reverse layer order: backward produces gradients from
the last layer to the first, so when conv k's filter gradient is done every
byte at offsets >= offset(conv k) is final and any bucket lying entirely in
that range is launched immediately (async), overlapping the remaining
backward kernels.  RCCL runs on its own stream and is ordered after the
engine stream's work at issue time; `finish` makes the engine stream wait
for every bucket before the optimizer.  The mean (1/world) is folded into
the optimizer launch as grad_scale.  Weights stay bitwise identical across
ranks because every rank applies the same update to the same reduced
gradient.
"""
from __future__ import annotations

import contextlib
from typing import List, Tuple

import torch
import torch.distributed as dist

DEFAULT_BUCKET_BYTES = 24 << 20


def make_buckets(layout, total: int, bucket_bytes: int = DEFAULT_BUCKET_BYTES) -> List[Tuple[int, int]]:
    """Contiguous [lo, hi) float ranges covering [0, total), cut at tensor
    starts, filled from the END (reverse layer order), each about
    bucket_bytes.  Returned in issue order (highest offsets first)."""
    starts = sorted(off for _, _, off, _ in layout)
    cap = max(1, bucket_bytes // 4)
    buckets = []
    hi = total
    acc_lo = total
    for off in reversed(starts):
        acc_lo = off
        if hi - acc_lo >= cap:
            buckets.append((acc_lo, hi))
            hi = acc_lo
    if hi > 0:
        buckets.append((0, hi))
    return buckets


class BucketAllReduce:
    """Per-step state machine: begin() -> param_ready(offset)* -> finish()."""

    def __init__(self, engine, world: int, bucket_bytes: int = DEFAULT_BUCKET_BYTES, group=None):
        self.eng = engine
        self.world = world
        self.group = group
        self.buckets = make_buckets(engine.layout, engine.nparam, bucket_bytes)
        self.works = []
        self.next = 0

    def begin(self, eng=None) -> None:
        self.works = []
        self.next = 0

    def _stream_ctx(self):
        s = getattr(self.eng, "stream", None)
        return torch.cuda.stream(s) if s is not None else contextlib.nullcontext()

    def _issue_ready(self, ready_from: int) -> None:
        eng = self.eng
        while self.next < len(self.buckets) and self.buckets[self.next][0] >= ready_from:
            lo, hi = self.buckets[self.next]
            with self._stream_ctx():
                w = dist.all_reduce(eng.grads[lo:hi], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            self.works.append(w)
            self.next += 1

    def param_ready(self, offset: int) -> None:
        """Called by Engine.backward after conv k's gradients are enqueued;
        every gradient at offsets >= offset is then final."""
        self._issue_ready(offset)

    def finish(self, eng=None) -> float:
        self._issue_ready(0)
        with self._stream_ctx():
            for w in self.works:
                w.wait()
        self.works = []
        return 1.0 / self.world
