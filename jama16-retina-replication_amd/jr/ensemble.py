"""Grouped ensemble inference: every member of an evaluate.py -lm ensemble in
ONE launch per layer.

The reference restores and runs each ensemble member in turn
(evaluate.py:166-211), and jr.Engine runs one member per engine.  At the
eval batch of 32 (evaluate.py:25) most GEMMs of one member are too small to
fill the 256 CUs (the 8x8 layers are M = 2,048 GEMMs), so members' forwards
were underfilled launches one after another.  EnsembleEngine keeps M members
resident as ONE replica with a member dimension: every tensor is member-major
([member][batch ...], fixed member strides), and each layer is

  * one grouped conv + BN-statistics launch (jr_conv2d_fwd_bn_stats_grouped:
    member = blockIdx.y, each with its own weights and statistics);
  * one grouped BN+ReLU apply per conv2d_bn layer (jr_bn_relu_apply_grouped);
  * pools and the global average pool over M x B images (the member-major
    activation buffers are simply a batch of M x B images);
  * the dense / sigmoid head per member (tiny).

Every member sees exactly its own batch-statistics BN (App. C Q1) and the
per-member tile plan, so its predictions are BITWISE those of a jr.Engine of
that member (tests/test_gpu_ensemble.py).  Inference only (train=False).
"""
from __future__ import annotations

import ctypes
import os
import weakref
from typing import List, Optional

import numpy as np
import torch

from . import _ffi
from .engine import DTYPES, fusable_pools, pinned_tile_table
from .inception import BN_EPS, build_inception_v3
from .lanes import Call, node_lanes, schedule
from .plan import build_plan


class EnsembleEngine:
    """M inference replicas (ensemble members) of one geometry on one GPU."""

    def __init__(self, params: List[np.ndarray], batch: int, height: int = 299, width: int = 299, units: int = 1,
                 device: int | torch.device = 0, dtype: str = "f32", conv_math: Optional[str] = None,
                 tiles: str = "pinned", head: str = "sigmoid", fuse_pool: Optional[bool] = None, lanes: int = 2):
        if dtype not in DTYPES:
            raise ValueError(f"dtype must be one of {sorted(DTYPES)}")
        if conv_math is None:
            conv_math = "x8" if dtype == "f32" else "bf16"
        if (dtype == "f32" and conv_math not in ("x8", "x6h", "f32")) or (dtype == "bf16" and conv_math != "bf16"):
            raise ValueError("grouped conv math: 'x8', 'x6h' or 'f32' for dtype f32, 'bf16' for dtype bf16")
        if not torch.cuda.is_available():
            raise RuntimeError("jr.EnsembleEngine needs a ROCm GPU (libjr has no CPU path)")
        if not params:
            raise ValueError("at least one member")
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        _ffi.init(self.device.index or 0)
        self.lib = _ffi.load()
        self.g = build_inception_v3(height, width, units)
        self.units = self.g.units
        self.plan = build_plan(self.g, True)
        if fuse_pool is None:            # (as jr.Engine: JR_FUSE_POOL=0 keeps the separate apply + max-pool)
            fuse_pool = os.environ.get("JR_FUSE_POOL", "1") != "0"
        # the stem's BN + ReLU inside its max-pools, every member in one launch
        self.pool_fused = fusable_pools(self.g, self.plan) if fuse_pool else {}
        self.cunits = self.plan.units
        self.nparam = self.plan.nparam
        self.members = len(params)
        self.batch = int(batch)
        self.dtype, self.dt = dtype, DTYPES[dtype]
        self.conv_math = conv_math
        self.cdt = {"x8": _ffi.JR_F32_X8, "x6h": _ffi.JR_F32_X6H}.get(conv_math, self.dt)
        self.x6h = conv_math == "x6h"
        self.esz = 2 if self.dt == _ffi.JR_BF16 else 4
        self.head_mode = _ffi.JR_HEAD_SIGMOID if head == "sigmoid" else _ffi.JR_HEAD_SOFTMAX
        self.stream = torch.cuda.Stream(device=self.device)
        self._s = ctypes.c_void_p(self.stream.cuda_stream)
        # branch lanes (jr.lanes, as jr.Engine): lane 0 is self.stream; every
        # lane has its OWN conv workspace (split-K slabs, stream-K partial
        # slots, statistics partials), declared as the resource ("ws", lane)
        self.nlanes = max(1, int(lanes))
        self.lane_streams = [self.stream] + [torch.cuda.Stream(device=self.device) for _ in range(1, self.nlanes)]
        self._fork_ev = torch.cuda.Event()
        self._join_ev = [torch.cuda.Event() for _ in range(self.nlanes - 1)]
        self._tail_ev = [torch.cuda.Event() for _ in range(self.nlanes)]
        self.precise_waits = os.environ.get("JR_PRECISE_WAITS", "1") != "0"   # (jr.Engine)
        self._prod_ev = {}               # libjr events (jr_event_create), as jr.Engine's
        self._lane_s = [ctypes.c_void_p(st.cuda_stream) for st in self.lane_streams]
        self._alloc()
        self.load_params(params)
        self.tiles = "heuristic"
        if tiles == "pinned":
            t = pinned_tile_table(conv_math, self.batch, height, width, False)
            if t is not None and all(u.name in t["configs"] for u in self.cunits):
                self._apply_configs(t["configs"])
                self.tiles = "pinned"
        elif tiles != "heuristic":
            raise ValueError("tiles: 'pinned' or 'heuristic'")
        self._gen = self.lib.jr_conv2d_config_generation()
        self._calls = {}

    # ------------------------------------------------------------------ memory
    def _t(self, n: int, dtype=torch.float32) -> torch.Tensor:
        return torch.zeros(int(n), dtype=dtype, device=self.device)

    def _alloc(self) -> None:
        g, B, M = self.g, self.batch, self.members
        at = torch.bfloat16 if self.dt == _ffi.JR_BF16 else torch.float32
        q = 8 if self.dt == _ffi.JR_BF16 else 4
        self.in_stride = (g.bufs[g.input_buf].c + q - 1) // q * q
        # member stride of every activation buffer: one member's B images
        self.act_ms = [B * b.h * b.w * (self.in_stride if b.id == g.input_buf else b.c) for b in g.bufs]
        self.acts = [self._t(M * n, at) for n in self.act_ms]
        self.raw_ms = {u.first.idx: B * u.ho * u.wo * u.cout for u in self.cunits}
        self.raw_unit = {k: self._t(M * n, at) for k, n in self.raw_ms.items()}
        self.stats_ms = 2 * sum(u.cout for u in self.cunits)
        self.stats = self._t(M * self.stats_ms)
        self.stat_off, off = {}, 0
        for u in self.cunits:
            self.stat_off[u.first.idx] = off
            off += 2 * u.cout
        feat_c = g.bufs[g.output_buf].c
        self.feat = self._t(M * B * feat_c)
        self.logits = self._t(M * B * self.units)
        self.probs = self._t(M * B * self.units)
        self.labels = self._t(B * self.units)
        self.loss = self._t(4 * M)
        self.params = self._t(M * self.nparam)
        if self.dt == _ffi.JR_BF16:
            # the bf16 W^T operand copies of every member (weights never change
            # in inference: prepared once, at load_params)
            layers, tiles, to = [], 0, 0
            self.wb_t_off = {}
            per = []
            for u in self.cunits:
                c8 = (u.cin + 7) // 8 * 8
                per.append((u, to, tiles))
                self.wb_t_off[u.first.idx] = to
                tiles += self.lib.jr_conv_weights_bf16_tiles(u.kh, u.kw, u.cin, u.cout)
                to += u.cout * u.kh * u.kw * c8
            self.wt_ms = (to + 7) // 8 * 8
            for m in range(M):
                for u, o, t0 in per:
                    layers.append(_ffi.WPrep(m * self.nparam + u.koff, 0, m * self.wt_ms + o, u.kh, u.kw, u.cin,
                                             u.cout, m * tiles + t0, 0))
            arr = (_ffi.WPrep * len(layers))(*layers)
            self.wprep_table = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(self.device)
            self.wprep_layers, self.wprep_tiles = len(layers), M * tiles
            self.w_t = self._t(M * self.wt_ms, torch.bfloat16)
        if self.x6h:
            # JR_F32_X6H magnitude words: 64 floats per (launch, member), the
            # members of a launch contiguous (the grouped conv's convention);
            # the filters never change in inference: measured at load_params
            U = len(self.cunits)
            self.absmax = self._t(64 * (U * M + 1))
            self._arow = {u.first.idx: k for k, u in enumerate(self.cunits)}
            nmax = max(B * u.ho * u.wo for u in self.cunits)
            self.act_bound = float(2 ** int(np.ceil(np.log2(np.sqrt(nmax) + 1024))))   # as jr.Engine
            segs = [_ffi.AbsmaxSeg(m * self.nparam + u.koff, u.kh * u.kw * u.cin * u.cout, k * M + m, 0.0)
                    for k, u in enumerate(self.cunits) for m in range(M)]
            segs += [_ffi.AbsmaxSeg(m * self.nparam + self.plan.poff[f"batch_normalization_{n.idx + 1}/beta"],
                                    n.cout, U * M, self.act_bound)
                     for m in range(M) for u in self.cunits for n in u.members]
            arr = (_ffi.AbsmaxSeg * len(segs))(*segs)
            self.absmax_table = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(self.device)
            self.absmax_nseg = len(segs)
        ws = 0
        for u in self.cunits:
            d = self._conv_desc(u, B)
            ws = max(ws, self.lib.jr_conv2d_workspace_size_grouped(ctypes.byref(d), self.cdt, M))
        self.ws_bytes = int(ws)
        self.ws_lane = [self._t((self.ws_bytes + 15) // 4 + 4) for _ in range(self.nlanes)]
        self.ws = self.ws_lane[0]

    def load_params(self, params: List[np.ndarray]) -> None:
        """Keras-layout flat parameters of every member (jr.checkpoint.load)."""
        if len(params) != self.members:
            raise ValueError(f"expected {self.members} members' parameters, got {len(params)}")
        with torch.cuda.stream(self.stream):     # ordered before the weight prep below
            for m, flat in enumerate(params):
                self.params[m * self.nparam:(m + 1) * self.nparam].copy_(
                    torch.from_numpy(self.plan.to_internal(self.g, flat)).to(self.device))
        if self.dt == _ffi.JR_BF16:
            with torch.cuda.stream(self.stream):
                _ffi.check("wprep", self.lib.jr_conv_weights_bf16_multi(
                    self.wprep_table.data_ptr(), self.wprep_layers, self.wprep_tiles, self.params.data_ptr(), None,
                    self.w_t.data_ptr(), self._s))
        if self.x6h:
            _ffi.check("absmax_prep", self.lib.jr_absmax_prep(
                self.params.data_ptr(), self.absmax_table.data_ptr(), self.absmax_nseg, self.absmax.data_ptr(),
                self.absmax.numel(), self._s))
        self.stream.synchronize()
        if self.x6h:
            _ffi.device_check()       # the beta guard of the activation bound (jr.h jr_absmax_prep)

    # ------------------------------------------------------------ descriptors
    def _conv_desc(self, u, B: int) -> _ffi.ConvDesc:
        xs = self.in_stride if u.x == self.g.input_buf else u.cin
        d = _ffi.ConvDesc(B, u.h, u.w, u.cin, u.cout, u.kh, u.kw, u.stride, u.stride,
                          u.pad_h, u.pad_w, u.ho, u.wo, 0, xs, 0, u.cout)
        if getattr(self, "x6h", False) and hasattr(self, "absmax"):
            d.x_bound = 1.0 if u.x == self.g.input_buf else self.act_bound
            d.w_absmax = self.absmax.data_ptr() + 4 * 64 * self._arow[u.first.idx] * self.members
        return d

    def _apply_configs(self, cfgs: dict) -> None:
        """The per-member forward tile of every launch (the eval table's)."""
        self._cfgs = cfgs
        for u in self.cunits:
            d = self._conv_desc(u, self.batch)
            _ffi.check("set_config", self.lib.jr_conv2d_set_config(ctypes.byref(d), _ffi.JR_CONV_FWD, self.cdt, 0,
                                                                   cfgs[u.name][0]))

    def _p(self, m: int, name: str) -> int:
        return self.params.data_ptr() + 4 * (m * self.nparam + self.plan.poff[name])

    # ------------------------------------------------------------- call list
    def _build_calls(self, B: int):
        if getattr(self, "_cfgs", None) is not None and self.lib.jr_conv2d_config_generation() != self._gen:
            self._apply_configs(self._cfgs)        # another caller moved this geometry's tiles
            self._calls.clear()
            self._gen = self.lib.jr_conv2d_config_generation()
        if B in self._calls:
            return self._calls[B]
        if B > self.batch or B <= 0:
            raise ValueError(f"batch {B} outside 1..{self.batch}")
        L, g, M, nl = self.lib, self.g, self.members, self.nlanes
        S = [ctypes.c_void_p(st.cuda_stream) for st in self.lane_streams]
        WS = [ctypes.c_void_p(w.data_ptr()) for w in self.ws_lane]
        wsb = ctypes.c_size_t(self.ws_bytes)
        lane_of = node_lanes(g, self.plan, nl)
        calls, keep = [], []

        def add(fn, args, name, lane, reads, writes):
            calls.append(Call(fn, args, name, lane, tuple(reads), tuple(writes)))

        # resources (jr.lanes.schedule), as jr.Engine: activation channel
        # slices, a launch's raw output + statistics, the lane's workspace
        slices = {g.input_buf: {0}}
        for n in g.nodes:
            slices.setdefault(n.y.buf, set()).add(n.y.c_off)
        a_all = lambda b: [("a", b, o) for o in sorted(slices[b])]  # noqa: E731
        A = lambda bid: self.acts[bid].data_ptr()  # noqa: E731
        fused_bufs = set(self.pool_fused.values())
        for i, n in enumerate(g.nodes):
            ln = lane_of[i]
            s = S[ln]
            if n.kind == "conv":
                u = self.plan.unit_of[n.idx]
                if u.first is not n:
                    continue
                d = self._conv_desc(u, B)
                keep.append(d)
                uid = u.first.idx
                so = self.stat_off[uid]
                if self.dt == _ffi.JR_BF16:
                    w, w_ms = self.w_t.data_ptr() + 2 * self.wb_t_off[uid], self.wt_ms
                else:
                    w, w_ms = self.params.data_ptr() + 4 * u.koff, self.nparam
                raw = self.raw_unit[uid].data_ptr()
                mean = self.stats.data_ptr() + 4 * so
                inv = mean + 4 * u.cout
                add(L.jr_conv2d_fwd_bn_stats_grouped,
                    (ctypes.byref(d), self.cdt, M, A(u.x), self.act_ms[u.x], w, w_ms, raw, self.raw_ms[uid], BN_EPS,
                     mean, inv, self.stats_ms, WS[ln], wsb, s), "conv_fwd", ln, a_all(u.x), [("r", uid), ("ws", ln)])
                rows = B * u.ho * u.wo
                for mem, co in zip(u.members, u.col_off):
                    if mem.y.buf in fused_bufs:
                        continue        # applied inside its max-pool
                    yb = g.bufs[mem.y.buf]
                    add(L.jr_bn_relu_apply_grouped,
                        (self.dt, M, raw, co, u.cout, self.raw_ms[uid], rows, mem.cout, mean + 4 * co, inv + 4 * co,
                         self.stats_ms, self._p(0, f"batch_normalization_{mem.idx + 1}/beta"), self.nparam,
                         A(mem.y.buf), mem.y.c_off, yb.c, self.act_ms[mem.y.buf], s), "bn_relu", ln,
                        [("r", uid)], [("a", mem.y.buf, mem.y.c_off)])
            else:
                # pools: the member-major buffers of a full batch are one
                # batch of M * B images (one launch); a partial last batch
                # (B < planned: members sit `batch` images apart) runs per member
                yb = g.bufs[n.y.buf]
                full = B == self.batch
                for m in range(1 if full else M):
                    d = _ffi.PoolDesc(M * B if full else B, n.h, n.w, n.c, n.ho, n.wo, 0, n.c, n.y.c_off, yb.c)
                    keep.append(d)
                    xi = A(n.x) + self.esz * m * self.act_ms[n.x]
                    yo = A(n.y.buf) + self.esz * m * self.act_ms[n.y.buf]
                    out = [("a", n.y.buf, n.y.c_off)]
                    if i in self.pool_fused:    # BN + ReLU of the producing layer on the fly
                        pn = next(q for q in g.nodes if q.y.buf == n.x)
                        puid = self.plan.unit_of[pn.idx].first.idx
                        so = self.stat_off[puid]
                        mean = self.stats.data_ptr() + 4 * (so + m * self.stats_ms)
                        add(L.jr_bn_relu_maxpool3x3s2_fwd_grouped,
                            (ctypes.byref(d), self.dt, B, self.raw_unit[puid].data_ptr()
                             + self.esz * m * self.raw_ms[puid], mean, mean + 4 * pn.cout, self.stats_ms,
                             self._p(m, f"batch_normalization_{pn.idx + 1}/beta"), self.nparam, yo, None, s),
                            "bn_relu_maxpool_fwd", ln, [("r", puid)], out)
                    elif n.kind == "maxpool":
                        add(L.jr_maxpool3x3s2_fwd, (ctypes.byref(d), self.dt, xi, yo, None, s), "maxpool_fwd", ln,
                            a_all(n.x), out)
                    else:
                        add(L.jr_avgpool3x3s1_fwd, (ctypes.byref(d), self.dt, xi, yo, s), "avgpool_fwd", ln,
                            a_all(n.x), out)
        ob = g.bufs[g.output_buf]
        s0 = S[0]
        if B == self.batch:
            add(L.jr_gap_fwd, (self.dt, A(g.output_buf), M * B, ob.h * ob.w, ob.c, self.feat.data_ptr(), s0),
                "gap_fwd", 0, a_all(g.output_buf), [("feat",)])
        else:
            for m in range(M):
                add(L.jr_gap_fwd, (self.dt, A(g.output_buf) + self.esz * m * self.act_ms[g.output_buf], B,
                                   ob.h * ob.w, ob.c, self.feat.data_ptr() + 4 * m * self.batch * ob.c, s0),
                    "gap_fwd", 0, a_all(g.output_buf), [("feat",)])
        for m in range(M):
            f = self.feat.data_ptr() + 4 * m * self.batch * ob.c
            o = 4 * m * self.batch * self.units
            add(L.jr_head_fwd, (self.head_mode, f, self._p(m, "dense/kernel"), self._p(m, "dense/bias"),
                                self.labels.data_ptr(), B, ob.c, self.units, self.logits.data_ptr() + o,
                                self.probs.data_ptr() + o, self.loss.data_ptr() + 16 * m, s0), "head_fwd", 0,
                [("feat",)], [("head",)])
        schedule(calls)
        self._calls[B] = (calls, keep)
        return self._calls[B]

    # ------------------------------------------------------------------- runs
    def set_batch(self, images, labels=None) -> int:
        """One batch for every member (NHWC uint8 or float32, host or device)."""
        B = int(images.shape[0])
        if B > self.batch or B <= 0:
            raise ValueError(f"batch {B} outside 1..{self.batch}")
        ib = self.g.bufs[self.g.input_buf]
        if tuple(images.shape[1:]) != (ib.h, ib.w, ib.c):
            raise ValueError(f"images must be [B,{ib.h},{ib.w},{ib.c}] NHWC, got {tuple(images.shape)}")
        with torch.cuda.stream(self.stream):
            x = torch.as_tensor(images)
            pixels = B * ib.h * ib.w
            dst = self.acts[self.g.input_buf]
            if x.dtype == torch.uint8:
                xd = x.to(self.device, non_blocking=True).reshape(-1)
                _ffi.check("jr_image_u8_to_nhwc", self.lib.jr_image_u8_to_nhwc(
                    xd.data_ptr(), dst.data_ptr(), self.dt, pixels, ib.c, self.in_stride, self._s))
                self._keep_u8 = xd
            else:
                v = dst[:pixels * self.in_stride].view(pixels, self.in_stride)
                v[:, ib.c:].zero_()
                v[:, :ib.c].copy_(x.to(torch.float32).reshape(pixels, ib.c).to(self.device, non_blocking=True))
            # every member reads the same images: copy member 0's
            n, k = self.act_ms[self.g.input_buf], pixels * self.in_stride
            for m in range(1, self.members):
                dst[m * n:m * n + k].copy_(dst[:k])
            if labels is not None:
                y = torch.as_tensor(labels, dtype=torch.float32).reshape(-1)
                self.labels[:y.numel()].copy_(y, non_blocking=True)
        return B

    def forward(self, B: Optional[int] = None) -> None:
        calls, _ = self._build_calls(B or self.batch)
        if self.nlanes > 1:          # fork: every lane after the batch upload on lane 0
            self._fork_ev.record(self.stream)
            for st in self.lane_streams[1:]:
                st.wait_event(self._fork_ev)
        for c in calls:
            st = self.lane_streams[c.lane]
            if self.precise_waits:
                for _, j in c.pwaits:    # the producing call on the other lane (jr.lanes.schedule)
                    # (one call list: producers always ran first)
                    _ffi.check("jr_stream_wait_event", self.lib.jr_stream_wait_event(self._lane_s[c.lane],
                                                                                     self._prod_ev[j]))
            else:
                for lj in c.waits:       # the other lane's tail
                    ev = self._tail_ev[lj]
                    ev.record(self.lane_streams[lj])
                    st.wait_event(ev)
            rc = c.fn(*c.args)
            if rc:
                raise _ffi.JRError(c.name, rc, _ffi.last_error())
            if c.record and self.precise_waits:
                ev = self._prod_ev.get(c.idx)
                if ev is None:
                    ev = self._prod_ev[c.idx] = ctypes.c_void_p()
                    _ffi.check("jr_event_create", self.lib.jr_event_create(ctypes.byref(ev)))
                    weakref.finalize(self, self.lib.jr_event_destroy, ev)
                _ffi.check("jr_event_record", self.lib.jr_event_record(ev, self._lane_s[c.lane]))
        for ev, st in zip(self._join_ev, self.lane_streams[1:]):    # join onto lane 0
            ev.record(st)
            self.stream.wait_event(ev)

    def synchronize(self) -> None:
        self.stream.synchronize()
        _ffi.device_check()          # (jr.Engine.synchronize: device-side failures raise)

    def predictions(self, n: Optional[int] = None) -> np.ndarray:
        """[members, n, units] sigmoid (softmax) outputs of the last forward."""
        n = self.batch if n is None else n
        self.synchronize()
        p = self.probs.cpu().numpy().reshape(self.members, self.batch, self.units)
        return p[:, :n].copy()
