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
backward kernels.  At an issue point with work, a stream outside the
engine's lanes (the feed stream of the torch transport, the comm stream of
JrComm) waits for every lane's work so far (Engine.fence_lanes) and the
all-reduce is issued from it; the lanes themselves never wait for each other
or for the exchange until `finish` makes lane 0 wait for every bucket before
the optimizer (an issue point without a ready bucket costs nothing).  The mean (1/world) is folded into
the optimizer launch as grad_scale.  Weights stay bitwise identical across
ranks because every rank applies the same update to the same reduced
gradient.

Two transports, same bucket walk:
  * torch.distributed all_reduce (backend 'nccl' = RCCL; 'gloo' on CPU);
  * libjr's own RCCL communicator (JrComm: jr_comm_init / jr_allreduce_sum,
    include/jr.h) on a dedicated comm stream that waits for every lane at
    each bucket's issue point; lane 0 waits for the comm stream before the
    optimizer.
and two payloads: fp32 (default; the sum of fp32 gradients) or bf16 (43.5 MB
instead of 87.1 MB: each bucket cast to bf16, summed in bf16 by RCCL, cast
back; ranks stay identical, the sum carries bf16 rounding).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from . import _ffi

DEFAULT_BUCKET_BYTES = 24 << 20
# the last bucket becomes ready only when the whole backward is done (the
# stem's filter gradients come last), so nothing hides its all-reduce: it is
# cut down to at most this much (the stem + the first block heads, ~1.9 MB)
# and the rest of the remainder issues while the stem's backward still runs
# (profiles/r06_dp_world1_ab.txt: issue points at -15.4, -13.7, -8.8 and
# -0.02 ms of a 24 ms fp32 step with one 10.4 MB remainder bucket)
DEFAULT_TAIL_BYTES = 2 << 20


def make_buckets(layout, total: int, bucket_bytes: int = DEFAULT_BUCKET_BYTES,
                 tail_bytes: int = DEFAULT_TAIL_BYTES) -> List[Tuple[int, int]]:
    """Contiguous [lo, hi) float ranges covering [0, total), cut at tensor
    starts, filled from the END (reverse layer order), each about
    bucket_bytes; the final bucket (which starts at 0) is split so that it
    holds at most tail_bytes (when a tensor start allows it).  Returned in
    issue order (highest offsets first)."""
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
        cut = max((off for off in starts if 0 < off < hi and 4 * off <= tail_bytes), default=0)
        if tail_bytes > 0 and 4 * hi > tail_bytes and cut > 0:
            buckets.append((cut, hi))
            hi = cut
        buckets.append((0, hi))
    return buckets


def resolve_run_id(run_id: Optional[str] = None) -> str:
    """The id that tags the RCCL unique-id file of THIS job (jr_comm_init_file).

    It must differ from every earlier job's, or a rank may join an id file an
    earlier job left at the same path.  In order:
      * an explicit run_id;
      * a nonce rank 0 draws and broadcasts over an initialised
        torch.distributed group (unique per job and per restart);
      * the launcher's TORCHELASTIC_RUN_ID + TORCHELASTIC_RESTART_COUNT, but
        never torchrun's default id, the literal "none", which every job that
        passes no --rdzv-id shares;
    otherwise ValueError.  MASTER_ADDR:MASTER_PORT is not used: a fixed port
    repeats from job to job."""
    if run_id:
        return str(run_id)
    if dist.is_available() and dist.is_initialized():
        box = [os.urandom(16).hex() if dist.get_rank() == 0 else None]
        dist.broadcast_object_list(box, 0)
        return f"nonce-{box[0]}"
    rid = os.environ.get("TORCHELASTIC_RUN_ID", "")
    if rid and rid.lower() != "none":
        return f"{rid}#{os.environ.get('TORCHELASTIC_RESTART_COUNT', '0')}"
    raise ValueError("JrComm(uid_path=...) needs a run id unique to this job: pass run_id, initialise "
                     "torch.distributed (rank 0 broadcasts a nonce), or launch with an explicit "
                     "--rdzv-id (TORCHELASTIC_RUN_ID is 'none' by default)")


class JrComm:
    """libjr's RCCL communicator (one per process / GPU)."""

    def __init__(self, rank: int, world: int, device: int, uid: Optional[bytes] = None,
                 uid_path: Optional[str] = None, timeout_ms: int = 120000, run_id: Optional[str] = None):
        self.lib = _ffi.load()
        self.h = ctypes.c_void_p()
        if uid_path is not None:
            # the id file is tagged with the job's run id: a file an earlier job
            # left at uid_path is ignored; rank 0 removes the file once the
            # communicator exists (jr_comm_init_file)
            run_id = resolve_run_id(run_id)
            _ffi.check("jr_comm_init_file", self.lib.jr_comm_init_file(rank, world, uid_path.encode(),
                                                                        run_id.encode(), device, timeout_ms,
                                                                        ctypes.byref(self.h)))
        else:
            if uid is None or len(uid) != 128:
                raise ValueError("JrComm needs the 128-byte unique id of rank 0 (JrComm.unique_id())")
            buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
            _ffi.check("jr_comm_init", self.lib.jr_comm_init(rank, world, buf, device, ctypes.byref(self.h)))
        self.rank, self.world = rank, world

    @staticmethod
    def unique_id() -> bytes:
        buf = (ctypes.c_uint8 * 128)()
        _ffi.check("jr_comm_unique_id", _ffi.load().jr_comm_unique_id(buf))
        return bytes(buf)

    @classmethod
    def from_torch_group(cls, rank: int, world: int, device: int) -> "JrComm":
        """Bootstrap the id through an initialised torch.distributed group."""
        box = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, 0)
        return cls(rank, world, device, uid=box[0])

    def allreduce(self, ptr: int, n: int, dtype: int, stream) -> None:
        _ffi.check("jr_allreduce_sum", self.lib.jr_allreduce_sum(self.h, ctypes.c_void_p(ptr), n, dtype,
                                                                  ctypes.c_void_p(stream)))

    def close(self) -> None:
        if self.h:
            _ffi.check("jr_comm_destroy", self.lib.jr_comm_destroy(self.h))
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BucketAllReduce:
    """Per-step state machine: begin() -> param_ready(offset)* -> finish()."""

    def __init__(self, engine, world: int, bucket_bytes: int = DEFAULT_BUCKET_BYTES, group=None,
                 comm: Optional[JrComm] = None, payload: str = "f32"):
        if payload not in ("f32", "bf16"):
            raise ValueError("payload must be 'f32' or 'bf16'")
        self.eng = engine
        self.world = world
        self.group = group
        self.comm = comm
        self.payload = payload
        self.buckets = make_buckets(engine.layout, engine.nparam, bucket_bytes)
        if hasattr(engine, "set_flush_points"):   # deferred filter-gradient slabs reduced before each bucket
            engine.set_flush_points([lo for lo, _ in self.buckets])
        self.works = []
        self.next = 0
        dev = getattr(engine, "device", None)
        self.half = (torch.empty(engine.nparam, dtype=torch.bfloat16, device=dev or engine.grads.device)
                     if payload == "bf16" else None)
        if comm is not None:
            self.comm_stream = torch.cuda.Stream(device=engine.grads.device)
            self._done_ev = torch.cuda.Event()
        # torch transport: buckets are issued from a feed stream that waits
        # for every lane at the issue point (Engine.fence_lanes); the lanes
        # never wait for each other or for the all-reduce until finish()
        self.feed = (torch.cuda.Stream(device=engine.grads.device)
                     if comm is None and getattr(engine, "stream", None) is not None else None)
        self.fences = 0                 # issue points that fenced the lanes (one per issue point with work)
        # trace=True: timing events on the issuing stream right after each
        # fence (the bucket's gradients are final: its all-reduce can start)
        # and on lane 0 when the backward has been joined (finish); see
        # overlap_ms()
        self.trace = False
        self._tev: List[Tuple[str, object]] = []

    def begin(self, eng=None) -> None:
        self.works = []
        self.next = 0
        self.fences = 0
        self._tev = []

    def _mark(self, kind: str, stream) -> None:
        if self.trace and stream is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(stream)
            self._tev.append((kind, ev))

    def overlap_ms(self) -> List[float]:
        """After a traced step (trace=True) has completed: for each issue
        point, when its buckets could start relative to the end of the
        backward, in ms (negative: while the backward was still running --
        the all-reduce overlaps it)."""
        end = next((ev for k, ev in self._tev if k == "backward_end"), None)
        if end is None:
            return []
        end.synchronize()
        return [round(end.elapsed_time(ev), 3) for k, ev in self._tev if k == "ready"]

    def _stream_ctx(self):
        s = getattr(self.eng, "stream", None)
        return torch.cuda.stream(s) if s is not None else contextlib.nullcontext()

    def _feed_ctx(self):
        return torch.cuda.stream(self.feed) if self.feed is not None else contextlib.nullcontext()

    def _fence(self, stream) -> None:
        """`stream` waits for every gradient enqueued so far on any lane
        (no stream: a host-side replica, nothing to order)."""
        eng = self.eng
        if stream is not None:
            if hasattr(eng, "fence_lanes"):
                eng.fence_lanes(stream)
            else:
                ev = torch.cuda.Event()
                ev.record(eng.stream)
                stream.wait_event(ev)
        self.fences += 1

    def _cast(self, fn, src: int, dst: int, n: int, stream) -> None:
        _ffi.check(fn, getattr(_ffi.load(), fn)(ctypes.c_void_p(src), ctypes.c_void_p(dst), n,
                                                ctypes.c_void_p(stream)))

    def _issue_jr(self, lo: int, hi: int) -> None:
        eng, cs = self.eng, self.comm_stream
        g = eng.grads.data_ptr() + 4 * lo
        if self.half is None:
            self.comm.allreduce(g, hi - lo, _ffi.JR_F32, cs.cuda_stream)
        else:
            h = self.half.data_ptr() + 2 * lo
            self._cast("jr_cast_f32_to_bf16", g, h, hi - lo, cs.cuda_stream)
            self.comm.allreduce(h, hi - lo, _ffi.JR_BF16, cs.cuda_stream)
            self._cast("jr_cast_bf16_to_f32", h, g, hi - lo, cs.cuda_stream)

    def _issue_torch(self, lo: int, hi: int):
        eng = self.eng
        with self._feed_ctx():
            if self.half is None:
                return dist.all_reduce(eng.grads[lo:hi], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            st = self.feed.cuda_stream if self.feed is not None else 0
            self._cast("jr_cast_f32_to_bf16", eng.grads.data_ptr() + 4 * lo, self.half.data_ptr() + 2 * lo,
                       hi - lo, st)
            w = dist.all_reduce(self.half[lo:hi], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            return (w, lo, hi)

    def ready(self, ready_from: int) -> bool:
        """Whether param_ready(ready_from) issues at least one bucket."""
        return self.next < len(self.buckets) and self.buckets[self.next][0] >= ready_from

    def _issue_ready(self, ready_from: int) -> None:
        if not self.ready(ready_from):
            return                      # nothing to issue: no fence, no wait anywhere
        st = self.comm_stream if self.comm is not None else self.feed
        self._fence(st)
        self._mark("ready", st)
        while self.ready(ready_from):
            lo, hi = self.buckets[self.next]
            if self.comm is not None:
                self._issue_jr(lo, hi)
            else:
                self.works.append(self._issue_torch(lo, hi))
            self.next += 1

    def param_ready(self, offset: int) -> None:
        """Called by Engine.backward after conv k's gradients are enqueued;
        every gradient at offsets >= offset is then final."""
        self._issue_ready(offset)

    def finish(self, eng=None) -> float:
        self._mark("backward_end", getattr(self.eng, "stream", None))
        self._issue_ready(0)
        if self.comm is not None:
            self._done_ev.record(self.comm_stream)
            self.eng.stream.wait_event(self._done_ev)
            return 1.0 / self.world
        with self._stream_ctx():
            for w in self.works:
                if isinstance(w, tuple):
                    w, lo, hi = w
                    w.wait()
                    st = self.eng.stream.cuda_stream if getattr(self.eng, "stream", None) is not None else 0
                    self._cast("jr_cast_bf16_to_f32", self.half.data_ptr() + 2 * lo,
                               self.eng.grads.data_ptr() + 4 * lo, hi - lo, st)
                else:
                    w.wait()
        self.works = []
        return 1.0 / self.world
