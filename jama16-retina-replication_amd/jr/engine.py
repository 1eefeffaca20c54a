"""Executor for the Inception-v3 training step / inference on libjr kernels.

The reference runs one `sess.run([global_step, mean_xentropy, train_op,
update_brier])` per batch (train.py:231-232): forward of the 94 conv2d_bn
blocks, head + loss, backward, and 190 ApplyMomentum updates.  This module is
that step, MI355X-native:

* All device memory is planned once per (batch, resolution): one NHWC buffer
  per block output (concat-free slices), a raw pre-BN buffer per conv launch
  (kept for the BN backward), one gradient buffer per activation buffer, a
  flat fp32 parameter / gradient / momentum buffer (so one optimizer launch
  and one all-reduce bucket walk cover all 190 tensors).  PyTorch tensors are
  used only as owners of that memory; every op is a libjr C-ABI call.
* Conv launches follow jr.plan: sibling 1x1 layers reading one buffer run as
  one fused GEMM (their kernels stored side by side), each member keeping its
  own BN, beta and output slice.
* Calls are pre-bound (ctypes function + argument tuple) into call lists, so a
  step is a flat loop of C calls on one HIP stream, and the whole step can be
  captured into a HIP graph (jr_graph_*) and replayed.
* Data parallel: gradients are all-reduced (torch.distributed backend 'nccl' =
  RCCL over xGMI) in buckets issued during the backward pass, in reverse layer
  order, so communication overlaps the remaining backward kernels.
"""
from __future__ import annotations

import ctypes
import dataclasses
import json
import os
import weakref
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np
import torch

from . import _ffi
from .inception import BN_EPS, Graph, PoolNode, build_inception_v3
from .init import init_params
from .lanes import Call, node_lanes, schedule
from .plan import ConvUnit, build_plan

DTYPES = {"f32": _ffi.JR_F32, "bf16": _ffi.JR_BF16}


_PINNED = None


def fusable_pools(g: Graph, plan) -> Dict[int, int]:
    """max-pool node index -> its input buffer, for every max-pool whose
    input is the whole output of ONE single-member conv launch and read by
    nothing else (the stem's conv2d_3 and conv2d_5): BN + ReLU then run
    inside the pool (jr_bn_relu_maxpool3x3s2_fwd)."""
    out = {}
    for i, n in enumerate(g.nodes):
        if n.kind != "maxpool":
            continue
        prod = [m for m in g.nodes if m.y.buf == n.x]
        readers = [m for m in g.nodes if m.x == n.x]
        if len(prod) != 1 or len(readers) != 1 or prod[0].kind != "conv":
            continue
        u = plan.unit_of[prod[0].idx]
        if len(u.members) == 1 and prod[0].y.c_off == 0 and prod[0].cout == g.bufs[n.x].c:
            out[i] = n.x
    return out


def pinned_tile_table(conv_math: str, batch: int, height: int, width: int, train: bool) -> Optional[dict]:
    """The committed tile table (jr/tiles_mi355x.json) of this workload, or None."""
    global _PINNED
    if _PINNED is None:
        # (JR_TILE_TABLES: another table file, for A/B runs of re-tuned tables)
        env = os.environ.get("JR_TILE_TABLES")
        if env and not os.path.exists(env):
            raise FileNotFoundError(f"JR_TILE_TABLES={env}: no such tile table file")
        p = env or os.path.join(os.path.dirname(os.path.abspath(__file__)), "tiles_mi355x.json")
        _PINNED = json.load(open(p))["tables"] if os.path.exists(p) else []
    for t in _PINNED:
        if (t["conv_math"], t["batch"], t["height"], t["width"], t["train"]) == (conv_math, batch, height, width,
                                                                              train):
            return t
    return None


class Engine:
    """One model replica on one GPU (one process per GPU)."""

    def __init__(self, batch: int, height: int = 299, width: int = 299, units: int = 1,
                 device: int | torch.device = 0, dtype: str = "f32", train: bool = True,
                 optimizer: str = "nesterov", lr: float = 3e-3, momentum: float = 0.9,
                 head: str = "sigmoid", seed: int = 0, graph: Optional[Graph] = None,
                 autotune: bool = False, tiles: str = "pinned", fuse_siblings: bool = True, lanes: int = 2,
                 conv_math: Optional[str] = None, defer_wgrad: Optional[bool] = None, fuse_pool: Optional[bool] = None,
                 fold_stats: Optional[bool] = None):
        if dtype not in DTYPES:
            raise ValueError(f"dtype must be one of {sorted(DTYPES)}")
        if conv_math is None:            # fp32 default: x8 (fp32-accurate, on the bf16 matrix cores)
            conv_math = "x8" if dtype == "f32" else "bf16"
        if (dtype == "f32" and conv_math not in ("f32", "x8", "x8p", "x6h")) or (dtype == "bf16" and conv_math != "bf16"):
            raise ValueError("conv_math: 'x8', 'x8p', 'x6h' or 'f32' for dtype f32 (x8 = JR_F32_X8, x8p = JR_F32_X8P "
                             "on pre-split operand planes, x6h = JR_F32_X6H scaled fp16 split, f32 = fp32 MFMA); "
                             "'bf16' for dtype bf16")
        if not torch.cuda.is_available():
            raise RuntimeError("jr.Engine needs a ROCm GPU (libjr has no CPU path)")
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        _ffi.init(self.device.index or 0)
        self.lib = _ffi.load()
        self.g = graph or build_inception_v3(height, width, units)
        self.batch = batch
        self.dt = DTYPES[dtype]
        self.dtype = dtype
        # dtype code of the convolution calls: JR_F32_X8 keeps every tensor
        # fp32 and forms the GEMM products on the bf16 matrix cores from an
        # exact three-way split (jr.h); everything else runs self.dt
        self.conv_math = conv_math
        self.x8p = conv_math == "x8p"
        # JR_F32_X6H: every conv operand's power-of-two scale from its largest
        # magnitude -- filters and data gradients measured on the device
        # (jr_absmax_prep once per step, the BN backward's fused max), the
        # activations from the bound |relu(xhat + beta)| <= sqrt(N - 1) +
        # max |beta| (Samuelson), beta guarded on the device (jr.h)
        self.x6h = conv_math == "x6h"
        self.cdt = {"x8": _ffi.JR_F32_X8, "x8p": _ffi.JR_F32_X8P, "x6h": _ffi.JR_F32_X6H}.get(conv_math, self.dt)
        self.train_mode = train
        if optimizer not in ("nesterov", "momentum", "sgd", "adam"):
            raise ValueError(f"unknown optimizer {optimizer}")
        self.optimizer = optimizer
        self.lr = float(lr)
        self.momentum = float(momentum)
        # Adam (north-star extra; TF AdamOptimizer defaults): accum holds m;
        # beta1_power / beta2_power are fp32 variables initialised to beta1 /
        # beta2 and multiplied by them (fp32) after every step, as TF's
        # AdamOptimizer._finish does
        self.adam_b1, self.adam_b2, self.adam_eps, self.adam_t = 0.9, 0.999, 1e-8, 0
        self.adam_b1p, self.adam_b2p = np.float32(self.adam_b1), np.float32(self.adam_b2)
        self.head_mode = _ffi.JR_HEAD_SIGMOID if head == "sigmoid" else _ffi.JR_HEAD_SOFTMAX
        self.units = self.g.units
        # JR_LANE_PRIORITY="p0,p1,...": HIP stream priority per lane (lower =
        # higher priority). Default: lane 0 (the trunk) high for fp32 steps,
        # measured 0.1 ms/step faster over 6 interleaved rounds on two boxes
        # (profiles/r05_ab_prio_f32*.txt); all normal for bf16, where it
        # measured neutral. Priority moves no result: scheduling only.
        prio_def = "-1,0" if self.dt == _ffi.JR_F32 else ""
        prio = [int(v) for v in os.environ.get("JR_LANE_PRIORITY", prio_def).split(",") if v.strip()]
        prio += [0] * max(0, int(lanes) - len(prio))
        self.stream = torch.cuda.Stream(device=self.device, priority=prio[0])
        self._s = ctypes.c_void_p(self.stream.cuda_stream)
        # lanes (jr.lanes): lane 0 is self.stream, where every step starts and ends
        self.nlanes = max(1, int(lanes))
        self.lane_streams = [self.stream] + [torch.cuda.Stream(device=self.device, priority=prio[i])
                                             for i in range(1, self.nlanes)]
        self._lane_s = [ctypes.c_void_p(st.cuda_stream) for st in self.lane_streams]
        self._fork_ev = torch.cuda.Event()
        self._join_ev = [torch.cuda.Event() for _ in range(self.nlanes - 1)]
        self._tail_ev = [torch.cuda.Event() for _ in range(self.nlanes)]
        # eager runs: a cross-lane consumer waits for its producing call (an
        # event recorded right after it) instead of the other lane's tail
        # (JR_PRECISE_WAITS=0: tail waits, as captured graphs always use)
        self.precise_waits = os.environ.get("JR_PRECISE_WAITS", "1") != "0"
        self._join_each = os.environ.get("JR_DP_JOIN_EACH", "0") == "1"
        self._prod_ev: Dict[int, object] = {}
        # producer events: libjr's (no timing, no system-scope fence: cheaper
        # to record) or torch's (JR_LANE_EVENTS=torch, for A/B runs)
        self._native_ev = os.environ.get("JR_LANE_EVENTS", "native") != "torch"
        self._capturing = False
        # backward order per conv launch: the data gradient (the critical
        # path to the next layer's BN backward) before the filter gradient
        # (JR_DGRAD_FIRST=0: filter gradient first)
        self.dgrad_first = os.environ.get("JR_DGRAD_FIRST", "1") != "0"
        # a fused sibling launch's members' BN + ReLU in one launch
        # (JR_APPLY_MULTI=0: one launch per member, for A/B runs)
        self.apply_multi = os.environ.get("JR_APPLY_MULTI", "1") != "0"
        self._vw = 8 if dtype == "bf16" else 4          # channels per 16-byte vector (one launch: <= 256 per row)
        self.plan = build_plan(self.g, fuse_siblings)
        # conv2d_bn outputs read only by a max-pool (the stem's conv2d_3 and
        # conv2d_5): BN + ReLU run inside the pool (jr_bn_relu_maxpool3x3s2_fwd)
        # and the full-resolution activation is never written
        if fuse_pool is None:           # (JR_FUSE_POOL=0: the separate apply + max-pool, for A/B runs)
            fuse_pool = os.environ.get("JR_FUSE_POOL", "1") != "0"
        self.pool_fused = fusable_pools(self.g, self.plan) if fuse_pool else {}
        # the BN-statistics finalize folded into the BN apply for launches whose
        # partials are single-stage and at most JR_FOLD_MAX_P per channel
        # (jr_conv2d_fwd_bn_partials + jr_bn_relu_apply_stats: a kernel
        # boundary fewer per layer; bitwise the separate finalize).  Opt-in
        # (JR_FOLD_STATS=1): measured neutral, f32 and bf16
        # (profiles/r05_ab_rows_{bf16,f32}.txt)
        if fold_stats is None:
            fold_stats = os.environ.get("JR_FOLD_STATS", "0") == "1"
        self.fold_stats = bool(fold_stats)
        self.fold_max_p = int(os.environ.get("JR_FOLD_MAX_P", "512"))
        self.cunits: List[ConvUnit] = self.plan.units
        self.layout, self.nparam = self.plan.layout, self.plan.nparam
        self._alloc()
        self.load_params(init_params(self.g, seed))
        self._calls: Dict[int, Tuple[list, list, list]] = {}
        self._retired: list = []        # call sets a captured graph may still reference
        # filter gradients of split-K wgrad GEMMs: slabs kept per layer and
        # summed by ONE jr_wgrad_reduce launch per flush point (the end of the
        # backward, and each gradient bucket's issue point: set_flush_points)
        # Default (None): deferred for bf16; fp32 reduces each layer's slabs
        # right after its filter-gradient GEMM (bitwise the same sums), which
        # with producer waits overlaps the other lane: 24.30 -> 24.06 ms per
        # step, bf16 9.25 -> 9.30 the other way (profiles/r05_ab_defer*.txt).
        # JR_DEFER_WGRAD=0/1 overrides the default.
        if defer_wgrad is None:
            env = os.environ.get("JR_DEFER_WGRAD", "")
            defer_wgrad = env == "1" if env in ("0", "1") else self.dt != _ffi.JR_F32
        self.defer_wgrad = bool(defer_wgrad)
        self._flush_points: List[int] = []
        self._graphs: Dict[int, int] = {}
        self.bucket_hooks: List[Tuple[int, Callable]] = []
        # conv tiles: "pinned" = the committed MI355X table for this workload
        # (jr/tiles_mi355x.json, tools/make_tile_tables.py) when there is one,
        # else the planner heuristic -- both deterministic, so every run on
        # every box sums in the same order; "autotune" (or autotune=True)
        # times the candidates on this box (fastest, box-dependent order)
        if tiles not in ("pinned", "heuristic", "autotune"):
            raise ValueError("tiles: 'pinned', 'heuristic' or 'autotune'")
        if autotune:
            tiles = "autotune"
        self.tiles = "heuristic"
        self.clear_tile_table()         # libjr's per-geometry overrides are process-wide
        if tiles == "autotune":
            self.autotune()
            self.tiles = "autotune"
        elif tiles == "pinned":
            t = pinned_tile_table(self.conv_math, self.batch, self.g.height, self.g.width, self.train_mode)
            if t is not None and all(u.name in t["configs"] for u in self.cunits):
                self.set_tile_table(t)
                self.tiles = "pinned"
        self._own_tiles()

    # ------------------------------------------------------------------ memory
    def _t(self, n: int, dtype=torch.float32) -> torch.Tensor:
        return torch.zeros(int(n), dtype=dtype, device=self.device)

    def _alloc(self) -> None:
        g, B = self.g, self.batch
        fl = torch.float32
        # activation dtype: fp32, or bf16 (parameters, gradients, momentum,
        # BN statistics and the head stay fp32 master copies either way)
        at = torch.bfloat16 if self.dt == _ffi.JR_BF16 else fl
        self.act_dtype = at
        self.esz = 2 if self.dt == _ffi.JR_BF16 else 4
        # the image buffer is kept one 16 B DMA piece wide per pixel (4 fp32 /
        # 8 bf16 channels, zeros past c = 3): conv1's c_in = 3 runs on libjr's
        # virtual channel padding
        q = 8 if self.dt == _ffi.JR_BF16 else 4
        self.in_stride = (g.bufs[g.input_buf].c + q - 1) // q * q
        self.acts = [self._t(B * b.h * b.w * (self.in_stride if b.id == g.input_buf else b.c), at)
                     for b in g.bufs]
        # raw (pre-BN) output and BN statistics per conv launch; a fused
        # group's members see channel slices of them
        self.raw_unit = {u.first.idx: self._t(B * u.ho * u.wo * u.cout, at) for u in self.cunits}
        self.stats = self._t(2 * sum(u.cout for u in self.cunits))
        self.raw, self.mean, self.invstd = {}, {}, {}
        self.mean_unit, self.invstd_unit = {}, {}
        off = 0
        for u in self.cunits:
            r = self.raw_unit[u.first.idx].view(B * u.ho * u.wo, u.cout)
            self.mean_unit[u.first.idx] = self.stats[off:off + u.cout]
            self.invstd_unit[u.first.idx] = self.stats[off + u.cout:off + 2 * u.cout]
            for n, co in zip(u.members, u.col_off):
                self.raw[n.idx] = r[:, co:co + n.cout]
                self.mean[n.idx] = self.stats[off + co:off + co + n.cout]
                self.invstd[n.idx] = self.stats[off + u.cout + co:off + u.cout + co + n.cout]
            off += 2 * u.cout
        self.argmax = {}
        for i, n in enumerate(g.nodes):
            if n.kind == "maxpool":
                self.argmax[i] = self._t(B * n.ho * n.wo * n.c, torch.uint8)
        feat_c = g.bufs[g.output_buf].c
        self.feat = self._t(B * feat_c)
        self.logits = self._t(B * self.units)
        self.probs = self._t(B * self.units)
        self.labels = self._t(B * self.units)
        self.loss = self._t(4)
        self.params = self._t(self.nparam)
        if self.train_mode:
            self.grads = self._t(self.nparam)
            self.accum = self._t(self.nparam)
            self.adam_v = self._t(self.nparam) if self.optimizer == "adam" else None
            self.dacts = [self._t(B * b.h * b.w * b.c, at) if b.id != g.input_buf else None
                          for b in g.bufs]
            # per-lane scratch for the raw-output gradient of the launch in flight
            self.draw_lane = [self._t(max(B * u.ho * u.wo * u.cout for u in self.cunits), at)
                              for _ in range(self.nlanes)]
            # the stem's filter gradients run on lane 1 beside its single-lane
            # data-gradient chain: a second raw-gradient buffer for lane 0 (the
            # next stem layer's BN backward must not overwrite what that
            # filter gradient still reads)
            self.draw_stem2 = (self._t(max(B * u.ho * u.wo * u.cout for u in self.cunits), at)
                               if self.nlanes > 1 and not self.x8p else None)
            self.draw = self.draw_lane[0]
            self.dfeat = self._t(B * feat_c)
            # the block-output BN backwards batched per block (jr_bn_relu_bwd_batch,
            # opt-in JR_BN_BATCH=1: bitwise the per-layer launch sets, measured
            # neutral -- bf16 9.343 -> 9.359, f32 24.85 -> 24.90 ms, the per-layer
            # sets already overlap on the two lanes): their raw gradients live in
            # two alternating sets of per-layer buffers
            self.bn_batch = (self._bn_batch_groups(B)
                             if not self.x8p and not self.x6h and os.environ.get("JR_BN_BATCH", "0") == "1" else [])
            slots = max((len(grp) for grp in self.bn_batch), default=0)
            self.drawb = [[self._t(max(B * grp[k].ho * grp[k].wo * grp[k].cout
                                       for grp in self.bn_batch if k < len(grp)), at) for k in range(slots)]
                          for _ in range(2 if slots else 0)]
        if self.dt == _ffi.JR_BF16 or self.x8p:
            self._alloc_bf16_filters(planes=3 if self.x8p else 1)
        if self.x8p:
            self._alloc_planes()
        ws = 0
        for u in self.cunits:
            d = self._conv_desc(u, B)
            ops = (_ffi.JR_CONV_FWD, _ffi.JR_CONV_BWD_DATA, _ffi.JR_CONV_BWD_FILTER)
            for op in (ops if self.train_mode else ops[:1]):
                ws = max(ws, self.lib.jr_conv2d_workspace_size(ctypes.byref(d), op, self.cdt))
            ws = max(ws, self.lib.jr_bn_workspace_size(B * u.ho * u.wo, u.cout))   # one backward per launch (or less)
        for grp in getattr(self, "bn_batch", []):        # one batched BN backward per block
            ws = max(ws, sum((self.lib.jr_bn_workspace_size(B * u.ho * u.wo, u.cout) + 255) // 256 * 256
                             for u in grp))
        for i in self.pool_fused:                      # the fused max-pool + BN backward's partials
            ws = max(ws, self.lib.jr_bn_relu_bwd_maxpool_workspace_size(ctypes.byref(self._pool_desc(g.nodes[i], B))))
        self.ws_bytes = int(ws)
        self.ws_lane = [self._t((self.ws_bytes + 15) // 4 + 4) for _ in range(self.nlanes)]
        # the stem filter gradients' own workspace on lane 1
        self.ws_stem = (self._t((self.ws_bytes + 15) // 4 + 4)
                        if self.train_mode and getattr(self, "draw_stem2", None) is not None else None)
        self.ws = self.ws_lane[0]
        if self.x6h:
            self._alloc_absmax(B)

    def _alloc_absmax(self, B: int) -> None:
        """JR_F32_X6H magnitude words: 64 floats per conv launch for its
        filter block (rows 0..U-1) and for its raw-output gradient (rows
        U..2U-1), and the jr_absmax_prep table (filters, then every BN beta
        with the activation guard)."""
        U = len(self.cunits)
        self.absmax = self._t(64 * 2 * U)
        self._arow = {u.first.idx: k for k, u in enumerate(self.cunits)}
        nmax = max(B * u.ho * u.wo for u in self.cunits)
        # activations are BN + ReLU outputs (or pools of them): |y| <= sqrt(N-1)
        # + max |beta|; bound = a power of two >= sqrt(N_max) + 1024, beta
        # guarded at that bound, so |y| <= 2 bound < the 4 bound the scale
        # keeps representable
        self.act_bound = float(2 ** int(np.ceil(np.log2(np.sqrt(nmax) + 1024))))
        segs = [_ffi.AbsmaxSeg(u.koff, u.kh * u.kw * u.cin * u.cout, k, 0.0) for k, u in enumerate(self.cunits)]
        for u in self.cunits:
            for m in u.members:
                off = self.plan.poff[f"batch_normalization_{m.idx + 1}/beta"]
                segs.append(_ffi.AbsmaxSeg(off, m.cout, 2 * U - 1, self.act_bound))
        # (the betas' maxima land in the last gradient row, zeroed again by
        # the same prep and raised by the first BN backward only after it:
        # harmless, a larger bound; conv2d_1's data gradient is never used)
        arr = (_ffi.AbsmaxSeg * len(segs))(*segs)
        self.absmax_table = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(self.device)
        self.absmax_nseg = len(segs)

    def _wmax(self, u: ConvUnit) -> int:
        return self.absmax.data_ptr() + 4 * 64 * self._arow[u.first.idx]

    def _dmax(self, u: ConvUnit) -> int:
        return self.absmax.data_ptr() + 4 * 64 * (len(self.cunits) + self._arow[u.first.idx])

    def _bn_batch_groups(self, B: int):
        """Conv launches whose BN backwards become due together: every member
        writes a slice of one block buffer (several producing launches: the
        branch-final layers of an Inception block), one launch set per launch
        (c / vector width <= 256), at most 512 reduce chunks (jr_bn.hip
        chunk_geom), not the stem's pooled layers; blocks with two or more."""
        g, vw = self.g, (8 if self.dt == _ffi.JR_BF16 else 4)
        producers: Dict[int, set] = {}
        for u in self.cunits:
            for m in u.members:
                producers.setdefault(m.y.buf, set()).add(u.first.idx)
        for n in g.nodes:
            if n.kind != "conv":
                producers.setdefault(n.y.buf, set()).add(("pool", id(n)))
        fused = set(self.pool_fused.values())
        groups: Dict[int, list] = {}
        for u in self.cunits:
            bufs = {m.y.buf for m in u.members}
            if len(bufs) != 1:
                continue
            buf = next(iter(bufs))
            M, c = B * u.ho * u.wo, u.cout
            tpr = c // vw
            rpp = max(1, 256 // tpr)
            step = rpp * 16
            rpc = -(-max(-(-M // 1024), step) // step) * step
            if (len(producers[buf]) < 2 or buf in fused or buf == g.output_buf or tpr > 256
                    or -(-M // rpc) > 512):
                continue
            groups.setdefault(buf, []).append(u)
        return [grp for grp in groups.values() if len(grp) >= 2]

    def _alloc_planes(self) -> None:
        """JR_F32_X8P operand planes (jr.h): the exact bf16 h/m/l split of
        every conv input buffer (written once per step by jr_split_x8p when
        the buffer is complete, read by the forward and the filter-gradient
        GEMMs) and of each lane's raw-output gradient scratch (dgrad and
        wgrad operand).  Channel radices are padded to 8 (the image: 3 -> 8)."""
        g, B = self.g, self.batch
        bf = torch.bfloat16
        self.plane_c = {}
        self.aplanes = {}
        for u in self.cunits:
            b = g.bufs[u.x]
            if u.x in self.aplanes:
                continue
            cp = (b.c + 7) // 8 * 8
            self.plane_c[u.x] = cp
            self.aplanes[u.x] = self._t(3 * B * b.h * b.w * cp, bf)
        if self.train_mode:
            n = max(B * u.ho * u.wo * u.cout for u in self.cunits)
            self.drawp_lane = [self._t(3 * n, bf) for _ in range(self.nlanes)]

    def _alloc_bf16_filters(self, planes: int = 1) -> None:
        """bf16 operand copies of every conv launch's kernel (block), refreshed
        from the fp32 master parameters by ONE jr_conv_weights_bf16_multi
        launch at the start of each forward: HWIO (bwd_data) and
        W^T [co][kh][kw][c8] (fwd).  planes = 3 (JR_F32_X8P): each copy is
        the three bf16 planes of the exact split, jr_conv_weights_x8p_multi."""
        L = self.lib
        self.wplanes = planes
        layers, tiles = [], 0
        self.wb_hwio_off, self.wb_t_off = {}, {}
        ho = to = 0
        for u in self.cunits:
            c8 = (u.cin + 7) // 8 * 8
            layers.append(_ffi.WPrep(u.koff, ho, to, u.kh, u.kw, u.cin, u.cout, tiles, 0))
            self.wb_hwio_off[u.first.idx], self.wb_t_off[u.first.idx] = ho, to
            tiles += L.jr_conv_weights_bf16_tiles(u.kh, u.kw, u.cin, u.cout)
            # 16 B-aligned starts (8 bf16); x8p: three planes per layer, plane
            # stride = the layer's element count (jr.h)
            hw_n = u.kh * u.kw * u.cin * u.cout
            ho += (planes * hw_n + 7) // 8 * 8
            to += planes * u.cout * u.kh * u.kw * c8
        arr = (_ffi.WPrep * len(layers))(*layers)
        self.wprep_table = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(self.device)
        self.wprep_layers, self.wprep_tiles = len(layers), tiles
        self.w_hwio = self._t(ho, torch.bfloat16)
        self.w_t = self._t(to, torch.bfloat16)

    def _wprep_call(self, stream=None):
        fn = self.lib.jr_conv_weights_x8p_multi if self.wplanes == 3 else self.lib.jr_conv_weights_bf16_multi
        return (fn,
                (self.wprep_table.data_ptr(), self.wprep_layers, self.wprep_tiles, self.params.data_ptr(),
                 self.w_hwio.data_ptr(), self.w_t.data_ptr(), stream or self._s), "wprep_bf16")

    def _wf(self, u: ConvUnit) -> int:
        """Filter operand of conv fwd: fp32 HWIO master block, or its bf16 W^T copy (planes)."""
        if self.dt == _ffi.JR_BF16 or self.x8p:
            return self.w_t.data_ptr() + 2 * self.wb_t_off[u.first.idx]
        return self.params.data_ptr() + 4 * u.koff

    def _wd(self, u: ConvUnit) -> int:
        """Filter operand of conv bwd_data: fp32 HWIO master block, or its bf16 copy (planes)."""
        if self.dt == _ffi.JR_BF16 or self.x8p:
            return self.w_hwio.data_ptr() + 2 * self.wb_hwio_off[u.first.idx]
        return self.params.data_ptr() + 4 * u.koff

    def autotune(self, progress: Optional[Callable[[str], None]] = None) -> None:
        """jr_conv2d_autotune every conv launch of the planned batch (cudnnFind
        style: times each tile configuration on this engine's own buffers and
        caches the fastest in libjr).  Runs before any data is loaded: it
        overwrites raw / gradient buffers."""
        L, B = self.lib, self.batch
        self._drop_calls()
        ws, wsb = ctypes.c_void_p(self.ws.data_ptr()), ctypes.c_size_t(self.ws_bytes)
        s = self._s
        if self.dt == _ffi.JR_BF16 or self.x8p:
            fn, args, name = self._wprep_call()
            _ffi.check(name, fn(*args))
        for u in self.cunits:
            if progress is not None:
                progress(u.name)
            d = self._conv_desc(u, B)
            x = (self.aplanes[u.x] if self.x8p else self.acts[u.x]).data_ptr()
            draw = (self.drawp_lane[0] if self.x8p else self.draw).data_ptr() if self.train_mode else 0
            raw = self.raw_unit[u.first.idx].data_ptr()
            _ffi.check("autotune fwd", L.jr_conv2d_autotune(ctypes.byref(d), _ffi.JR_CONV_FWD, self.cdt, x,
                                                             self._wf(u), raw, ws, wsb, s))
            if not self.train_mode:
                continue
            _ffi.check("autotune wgrad", L.jr_conv2d_autotune(
                ctypes.byref(d), _ffi.JR_CONV_BWD_FILTER, self.cdt, x, draw,
                self.grads.data_ptr() + 4 * u.koff, ws, wsb, s))
            if u.x != self.g.input_buf:
                _ffi.check("autotune dgrad", L.jr_conv2d_autotune(
                    ctypes.byref(d), _ffi.JR_CONV_BWD_DATA, self.cdt, draw, self._wd(u),
                    self.dacts[u.x].data_ptr(), ws, wsb, s))
        self.synchronize()
        if self.train_mode:
            self.grads.zero_()
        self._own_tiles()

    def conv_configs(self) -> dict:
        """{conv launch name: (fwd cfg, wgrad cfg, [dgrad cfg per phase])} in use."""
        out = {}
        for u in self.cunits:
            d = self._conv_desc(u, self.batch)
            f = self.lib.jr_conv2d_get_config(ctypes.byref(d), _ffi.JR_CONV_FWD, self.cdt, 0)
            wg = self.lib.jr_conv2d_get_config(ctypes.byref(d), _ffi.JR_CONV_BWD_FILTER, self.cdt, 0)
            dg = [self.lib.jr_conv2d_get_config(ctypes.byref(d), _ffi.JR_CONV_BWD_DATA, self.cdt, p)
                  for p in range(u.stride * u.stride)]
            out[u.name] = (f, wg, dg)
        return out

    def tile_table(self) -> dict:
        """The conv tile configuration of every launch, as saved in checkpoint
        meta (jr.checkpoint) and accepted back by set_tile_table: with the
        same table two runs sum in the same order (bitwise-equal steps on any
        MI355X).  Keyed by conv math, batch and resolution."""
        return {"conv_math": self.conv_math, "batch": self.batch, "height": self.g.height,
                "width": self.g.width, "configs": {k: [f, wg, list(dg)] for k, (f, wg, dg) in
                                                   self.conv_configs().items()}}

    def _drop_calls(self) -> None:
        """Forget the bound call lists (tile plans or flush points changed);
        their buffers stay alive for graphs captured from them."""
        self._retired.extend(self._calls.values())
        self._calls.clear()

    def set_flush_points(self, points) -> None:
        """Flat-gradient offsets at which a consumer (jr.dist.BucketAllReduce)
        needs every gradient at offsets >= the point final: the deferred
        filter-gradient slabs are reduced before the param_ready hook of the
        first launch whose offset is <= the point."""
        self._flush_points = sorted((int(p) for p in points), reverse=True)
        self._drop_calls()

    def set_tile_table(self, table: dict) -> None:
        """Pin every conv launch to the configs of `table` (tile_table())."""
        self._drop_calls()
        if (table.get("conv_math"), table.get("batch"), table.get("height"), table.get("width")) != \
                (self.conv_math, self.batch, self.g.height, self.g.width):
            raise ValueError("tile table is for another conv math / batch / resolution")
        self._apply_configs(table["configs"])
        self._own_tiles()

    def _own_tiles(self) -> None:
        """Record the configs this engine's call lists are bound to (libjr's
        overrides are process-wide: another engine or caller of the same
        geometry may change them; _ensure_tiles puts these back)."""
        if not hasattr(self, "tiles"):
            return                  # still in __init__ (clear_tile_table before the table is chosen)
        self._tile_cfgs = self.tile_table()["configs"]
        self._tile_gen = self.lib.jr_conv2d_config_generation()

    def _ensure_tiles(self) -> None:
        """Re-apply this engine's configs if libjr's overrides changed since it
        applied them (the deferred filter-gradient segments bind
        the split count of the plan at call-list build time)."""
        gen = self.lib.jr_conv2d_config_generation()
        if getattr(self, "_tile_cfgs", None) is None or gen == self._tile_gen:
            return
        self._apply_configs(self._tile_cfgs)     # the same plans the call lists were built with
        self._tile_gen = self.lib.jr_conv2d_config_generation()

    def _apply_configs(self, cfgs: dict) -> None:
        for u in self.cunits:
            f, wg, dg = cfgs[u.name]
            d = self._conv_desc(u, self.batch)
            _ffi.check("set_config", self.lib.jr_conv2d_set_config(ctypes.byref(d), _ffi.JR_CONV_FWD, self.cdt, 0, f))
            if not self.train_mode:
                continue
            _ffi.check("set_config", self.lib.jr_conv2d_set_config(ctypes.byref(d), _ffi.JR_CONV_BWD_FILTER,
                                                                   self.cdt, 0, wg))
            if u.x != self.g.input_buf:
                for p, c in enumerate(dg):
                    _ffi.check("set_config", self.lib.jr_conv2d_set_config(ctypes.byref(d), _ffi.JR_CONV_BWD_DATA,
                                                                           self.cdt, p, c))

    def clear_tile_table(self) -> None:
        """Back to the deterministic planner heuristic for every conv launch
        (drops autotuned or pinned configs of this engine's geometries)."""
        self._clear_configs()
        self._own_tiles()

    def _clear_configs(self) -> None:
        if hasattr(self, "_calls"):
            self._drop_calls()
        for u in self.cunits:
            d = self._conv_desc(u, self.batch)
            ops = [(_ffi.JR_CONV_FWD, 0)]
            if self.train_mode:
                ops.append((_ffi.JR_CONV_BWD_FILTER, 0))
                if u.x != self.g.input_buf:
                    ops += [(_ffi.JR_CONV_BWD_DATA, p) for p in range(u.stride * u.stride)]
            for op, p in ops:
                _ffi.check("set_config", self.lib.jr_conv2d_set_config(ctypes.byref(d), op, self.cdt, p, -1))

    # ------------------------------------------------------------ parameters
    def load_params(self, flat: np.ndarray) -> None:
        """Keras-layout flat parameters (jr.init.param_layout order)."""
        self.params.copy_(torch.from_numpy(self.plan.to_internal(self.g, flat)).to(self.device))
        if self.train_mode:
            self.accum.zero_()
            self.grads.zero_()
            # optimizer state restarts with the parameters: Adam's v slot and
            # its fp32 beta powers (TF initialises beta1_power / beta2_power to
            # beta1 / beta2 with the slots)
            if self.adam_v is not None:
                self.adam_v.zero_()
            self.adam_t = 0
            self.adam_b1p, self.adam_b2p = np.float32(self.adam_b1), np.float32(self.adam_b2)

    def params_numpy(self) -> np.ndarray:
        """Parameters in the Keras layout (checkpoints, the oracle)."""
        torch.cuda.synchronize(self.device)
        return self.plan.to_keras(self.g, self.params.cpu().numpy())

    def grads_numpy(self) -> np.ndarray:
        """Gradients of the last backward in the Keras layout."""
        torch.cuda.synchronize(self.device)
        return self.plan.to_keras(self.g, self.grads.cpu().numpy())

    def _p(self, name: str) -> int:
        return self.params.data_ptr() + 4 * self.plan.poff[name]

    def _gp(self, name: str) -> int:
        return self.grads.data_ptr() + 4 * self.plan.poff[name]

    # ------------------------------------------------------------ descriptors
    def _conv_desc(self, u: ConvUnit, B: int) -> _ffi.ConvDesc:
        if self.x8p:          # x describes the operand planes: channel radix padded to 8
            xs = (u.cin + 7) // 8 * 8
        else:
            xs = self.in_stride if u.x == self.g.input_buf else u.cin
        d = _ffi.ConvDesc(B, u.h, u.w, u.cin, u.cout, u.kh, u.kw, u.stride, u.stride,
                          u.pad_h, u.pad_w, u.ho, u.wo, 0, xs, 0, u.cout)
        if self.x6h and hasattr(self, "absmax"):
            d.x_bound = 1.0 if u.x == self.g.input_buf else self.act_bound    # images: f32(k) * f32(1/255) <= 1
            d.w_absmax = self._wmax(u)
            d.dy_absmax = self._dmax(u)
        return d

    def _pool_desc(self, n: PoolNode, B: int) -> _ffi.PoolDesc:
        yb = self.g.bufs[n.y.buf]
        return _ffi.PoolDesc(B, n.h, n.w, n.c, n.ho, n.wo, 0, n.c, n.y.c_off, yb.c)

    # ------------------------------------------------------------- call lists
    def _bn_groups(self, u: ConvUnit):
        """BN backward launch sets of a conv launch: all members at once while
        the launch's channels fit one 256-thread row (jr_bn: <= 256 vectors of
        4 fp32 / 8 bf16), else one set per member.  [(member, col_off), ...]"""
        groups = [list(zip(u.members, u.col_off))]
        if u.cout // (8 if self.dt == _ffi.JR_BF16 else 4) > 256:
            groups = [[mc] for mc in groups[0]]
        return groups

    def _build_calls(self, B: int, nl: Optional[int] = None, one_stream: bool = False):
        """Pre-bound Calls (jr.lanes) for forward, backward, update on nl
        lanes (default self.nlanes), with their cross-lane waits:
        (fwd, bwd, opt, keep, None).  one_stream: every call is bound to
        lane 0's stream (per-lane scratch kept) for the explicit-DAG graph
        capture, where the lanes become graph branches (capture())."""
        self._ensure_tiles()
        nl = self.nlanes if nl is None else max(1, min(int(nl), self.nlanes))
        key = (B, nl, one_stream)
        if key in self._calls:
            return self._calls[key]
        if B > self.batch or B <= 0:
            raise ValueError(f"batch {B} outside 1..{self.batch}")
        L, g, dt, cdt = self.lib, self.g, self.dt, self.cdt
        S = [ctypes.c_void_p(st.cuda_stream) for st in self.lane_streams[:nl]]
        if one_stream:
            S = [S[0]] * nl
        WS = [ctypes.c_void_p(w.data_ptr()) for w in self.ws_lane[:nl]]
        wsb = ctypes.c_size_t(self.ws_bytes)
        lane_of = node_lanes(g, self.plan, nl)
        keep = []  # keep ctypes structs alive
        fwd, bwd, opt, seq = [], [], [], []

        def add(lst, fn, args, name, lane, reads=(), writes=(), nbytes=0):
            c = Call(fn, args, name, lane, tuple(reads), tuple(writes), nbytes=int(nbytes))
            lst.append(c)
            seq.append(c)

        # resources (jr.lanes.schedule): activation / gradient channel slices
        slices: Dict[int, set] = {g.input_buf: {0}}
        for n in g.nodes:
            slices.setdefault(n.y.buf, set()).add(n.y.c_off)
        a_all = lambda b: [("a", b, o) for o in sorted(slices[b])]  # noqa: E731
        d_all = lambda b: [("d", b, o) for o in sorted(slices[b])]  # noqa: E731
        A = lambda bid: self.acts[bid].data_ptr()  # noqa: E731
        unit_of = self.plan.unit_of
        x8p = self.x8p
        wkey = ("w16",) if (dt == _ffi.JR_BF16 or x8p) else ("p",)
        if dt == _ffi.JR_BF16 or x8p:
            add(fwd, *self._wprep_call(S[0]), 0, [("p",)], [("w16",)])
        # x6h: the convs read their filters' magnitude words besides the filters
        xw = [("wmax",)] if self.x6h else []
        if self.x6h:
            # the filters' magnitudes (and the beta guard), and every
            # gradient row zeroed, before the first conv of the step
            add(fwd, L.jr_absmax_prep, (self.params.data_ptr(), self.absmax_table.data_ptr(), self.absmax_nseg,
                                        self.absmax.data_ptr(), self.absmax.numel(), S[0]), "absmax_prep", 0,
                [("p",)], [("wmax",)] + [("dmax", u.first.idx) for u in self.cunits], nbytes=4 * self.nparam)
        # x8p: conv operands are the split planes of the input buffer, written
        # once (by the lane of its first consumer) when the buffer is complete
        AX = (lambda bid: self.aplanes[bid].data_ptr()) if x8p else A  # noqa: E731
        ax_reads = (lambda bid: [("ap", bid)]) if x8p else a_all  # noqa: E731
        split_done = set()
        fused_bufs = set(self.pool_fused.values())
        for i, n in enumerate(g.nodes):
            ln = lane_of[i]
            s, ws = S[ln], WS[ln]
            if n.kind == "conv":
                u = unit_of[n.idx]
                if u.first is not n:
                    continue            # emitted with the group's first member
                d = self._conv_desc(u, B)
                keep.append(d)
                M = B * u.ho * u.wo
                uid = u.first.idx
                raw = self.raw_unit[uid].data_ptr()
                if x8p and u.x not in split_done:
                    split_done.add(u.x)
                    b = g.bufs[u.x]
                    cp = self.plane_c[u.x]
                    rows = B * b.h * b.w
                    src_stride = self.in_stride if u.x == g.input_buf else b.c
                    add(fwd, L.jr_split_x8p, (A(u.x), rows, b.c, 0, src_stride, AX(u.x), cp, 0, cp,
                                              self.batch * b.h * b.w * cp, s),
                        "split_x8p", ln, a_all(u.x), [("ap", u.x)], nbytes=rows * (4 * b.c + 6 * cp))
                lay = None
                if self.fold_stats and not any(m.y.buf in fused_bufs for m in u.members):
                    lay = _ffi.BnPartials()
                    _ffi.check("jr_conv2d_bn_partials_layout",
                               L.jr_conv2d_bn_partials_layout(ctypes.byref(d), cdt, ctypes.byref(lay)))
                    if not lay.single_stage or lay.P > self.fold_max_p:
                        lay = None
                if lay is not None:
                    # conv + the statistics partials; each member's BN apply
                    # combines its channels' partials (and stores mean / invstd)
                    add(fwd, L.jr_conv2d_fwd_bn_partials, (ctypes.byref(d), cdt, AX(u.x), self._wf(u), raw, ws, wsb,
                                                           s),
                        "conv_fwd", ln, ax_reads(u.x) + [wkey] + xw, [("r", uid), ("ws", ln)])
                    part = ws.value + lay.ws_offset
                    for m, co in zip(u.members, u.col_off):
                        yb = g.bufs[m.y.buf]
                        add(fwd, L.jr_bn_relu_apply_stats,
                            (dt, raw, co, u.cout, M, m.cout, part, lay.P, lay.R, u.cout, co, BN_EPS,
                             self.mean[m.idx].data_ptr(), self.invstd[m.idx].data_ptr(),
                             self._p(f"batch_normalization_{m.idx + 1}/beta"), A(m.y.buf), m.y.c_off, yb.c, s),
                            "bn_relu", ln, [("r", uid), ("ws", ln), ("p",)], [("a", m.y.buf, m.y.c_off), ("r", uid)],
                            nbytes=2 * M * m.cout * self.esz)
                    continue
                # conv + the BN batch statistics of its raw output, fused
                add(fwd, L.jr_conv2d_fwd_bn_stats, (ctypes.byref(d), cdt, AX(u.x), self._wf(u), raw, BN_EPS,
                                                    self.mean_unit[uid].data_ptr(),
                                                    self.invstd_unit[uid].data_ptr(), ws, wsb, s),
                    "conv_fwd", ln, ax_reads(u.x) + [wkey] + xw, [("r", uid), ("ws", ln)])
                if (self.apply_multi and len(u.members) > 1 and u.cout // self._vw <= 256
                        and not any(m.y.buf in fused_bufs for m in u.members)):
                    # every member's BN + ReLU in one launch (jr_bn_relu_apply_multi)
                    segs = (_ffi.BnApplySeg * len(u.members))(*[
                        _ffi.BnApplySeg(A(m.y.buf), m.y.c_off, g.bufs[m.y.buf].c, m.cout,
                                        self._p(f"batch_normalization_{m.idx + 1}/beta")) for m in u.members])
                    keep.append(segs)
                    add(fwd, L.jr_bn_relu_apply_multi, (dt, len(u.members), ctypes.byref(segs), raw, 0, u.cout, M,
                                                        u.cout, self.mean_unit[uid].data_ptr(),
                                                        self.invstd_unit[uid].data_ptr(), s),
                        "bn_relu", ln, [("r", uid), ("p",)], [("a", m.y.buf, m.y.c_off) for m in u.members],
                        nbytes=2 * M * u.cout * self.esz)
                    continue
                for m, co in zip(u.members, u.col_off):
                    if m.y.buf in fused_bufs:
                        continue        # applied inside its max-pool
                    yb = g.bufs[m.y.buf]
                    add(fwd, L.jr_bn_relu_apply, (dt, raw, co, u.cout, M, m.cout, self.mean[m.idx].data_ptr(),
                                                  self.invstd[m.idx].data_ptr(),
                                                  self._p(f"batch_normalization_{m.idx + 1}/beta"),
                                                  A(m.y.buf), m.y.c_off, yb.c, s),
                        "bn_relu", ln, [("r", uid), ("p",)], [("a", m.y.buf, m.y.c_off)],
                        nbytes=2 * M * m.cout * self.esz)
            elif n.kind == "maxpool" and i in self.pool_fused:
                d = self._pool_desc(n, B)
                pn = next(m for m in g.nodes if m.y.buf == n.x)          # the conv2d_bn layer it applies
                d.x_c_off, d.x_c_stride = 0, pn.cout                       # its raw output
                keep.append(d)
                puid = unit_of[pn.idx].first.idx
                add(fwd, L.jr_bn_relu_maxpool3x3s2_fwd, (ctypes.byref(d), dt, self.raw_unit[puid].data_ptr(),
                                                         self.mean[pn.idx].data_ptr(), self.invstd[pn.idx].data_ptr(),
                                                         self._p(f"batch_normalization_{pn.idx + 1}/beta"),
                                                         A(n.y.buf), self.argmax[i].data_ptr(), s),
                    "bn_relu_maxpool_fwd", ln, [("r", puid), ("p",)], [("a", n.y.buf, n.y.c_off), ("am", i)],
                    nbytes=B * n.c * (n.h * n.w * self.esz + n.ho * n.wo * (self.esz + 1)))
            elif n.kind == "maxpool":
                d = self._pool_desc(n, B)
                keep.append(d)
                add(fwd, L.jr_maxpool3x3s2_fwd, (ctypes.byref(d), dt, A(n.x), A(n.y.buf), self.argmax[i].data_ptr(), s),
                    "maxpool_fwd", ln, a_all(n.x), [("a", n.y.buf, n.y.c_off), ("am", i)],
                    nbytes=B * n.c * (n.h * n.w * self.esz + n.ho * n.wo * (self.esz + 1)))
            else:
                d = self._pool_desc(n, B)
                keep.append(d)
                add(fwd, L.jr_avgpool3x3s1_fwd, (ctypes.byref(d), dt, A(n.x), A(n.y.buf), s),
                    "avgpool_fwd", ln, a_all(n.x), [("a", n.y.buf, n.y.c_off)],
                    nbytes=B * n.c * (n.h * n.w + n.ho * n.wo) * self.esz)
        ob = g.bufs[g.output_buf]
        s0 = S[0]
        add(fwd, L.jr_gap_fwd, (dt, A(g.output_buf), B, ob.h * ob.w, ob.c, self.feat.data_ptr(), s0),
            "gap_fwd", 0, a_all(g.output_buf), [("feat",)])
        add(fwd, L.jr_head_fwd, (self.head_mode, self.feat.data_ptr(), self._p("dense/kernel"),
                                 self._p("dense/bias"), self.labels.data_ptr(), B, ob.c, self.units,
                                 self.logits.data_ptr(), self.probs.data_ptr(), self.loss.data_ptr(), s0),
            "head_fwd", 0, [("feat",), ("p",), ("lab",)], [("head",)])
        if self.train_mode:
            D = lambda bid: self.dacts[bid].data_ptr()  # noqa: E731
            # deferred filter gradients: per-layer slab regions of one arena
            defer: Dict[int, Tuple[_ffi.WgradSeg, int, int]] = {}
            if self.defer_wgrad:
                off = 0
                for u in self.cunits:
                    d = self._conv_desc(u, B)
                    keep.append(d)
                    sg = _ffi.WgradSeg()
                    _ffi.check("jr_conv2d_wgrad_seg", L.jr_conv2d_wgrad_seg(ctypes.byref(d), cdt, ctypes.byref(sg)))
                    if sg.splits > 1:
                        nb = 4 * sg.splits * sg.m * sg.n
                        sg.dw = self.grads.data_ptr() + 4 * u.koff
                        defer[u.first.idx] = (sg, off, nb)
                        off += (nb + 255) // 256 * 256
                arena = self._t(off // 4 + 64)
                keep.append(arena)
                for sg, o, _ in defer.values():
                    sg.slabs = arena.data_ptr() + o
                self.slab_bytes = off
            pending: List[Tuple[_ffi.WgradSeg, int]] = []
            flush_at = list(self._flush_points)

            def flush():
                """One jr_wgrad_reduce over every pending layer (lane 0)."""
                if not pending:
                    return
                arr = (_ffi.WgradSeg * len(pending))()
                blocks = 0
                for k, (sg, _) in enumerate(pending):
                    arr[k] = sg
                    arr[k].block0 = blocks
                    blocks += sg.blocks
                table = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(self.device)
                keep.append(table)
                nbytes = sum(4 * sg.m * sg.n * (sg.splits + 1) for sg, _ in pending)
                add(bwd, L.jr_wgrad_reduce, (table.data_ptr(), len(pending), blocks, S[0]), "wgrad_reduce", 0,
                    [("slab", uid) for _, uid in pending], [("g", uid) for _, uid in pending], nbytes=nbytes)
                pending.clear()
            add(bwd, L.jr_head_bwd, (self.head_mode, self.feat.data_ptr(), self._p("dense/kernel"),
                                     self.probs.data_ptr(), self.labels.data_ptr(), B, ob.c, self.units,
                                     self.dfeat.data_ptr(), self._gp("dense/kernel"), self._gp("dense/bias"), s0),
                "head_bwd", 0, [("feat",), ("p",), ("head",), ("lab",)], [("dfeat",), ("g", "dense")])
            add(bwd, L.jr_gap_bwd, (dt, self.dfeat.data_ptr(), B, ob.h * ob.w, ob.c, D(g.output_buf), s0),
                "gap_bwd", 0, [("dfeat",)], d_all(g.output_buf))
            written = set()
            # fp32: the fused stem pools' backward carries the BN reduce
            # (bf16 keeps the separate kernels, whose batch-of-rows fp32 sums
            # it would not reproduce bit for bit)
            pool_bwd = (self.pool_fused if dt == _ffi.JR_F32 and os.environ.get("JR_FUSE_POOL_BWD", "1") != "0"
                        else {})
            readers: Dict[int, int] = {}
            for q in g.nodes:
                readers[q.x] = readers.get(q.x, 0) + 1
            # the stem: the layers before the first buffer with several readers
            stem_end = next((j for j, q in enumerate(g.nodes) if readers[q.x] > 1), 0)
            stem_split = (nl > 1 and self.draw_stem2 is not None
                          and os.environ.get("JR_STEM_WGRAD_LANE", "1") != "0")
            sbuf = 0
            # batched block-output BN backwards: unit -> (group, slot); a group
            # is issued where its first unit comes up (its upstream gradients
            # are final there), on that unit's lane, into set `bset`
            in_batch = {u.first.idx: (gi, k) for gi, grp in enumerate(self.bn_batch) for k, u in enumerate(grp)}
            batch_draw: Dict[int, Tuple[int, Tuple]] = {}   # uid -> (raw-gradient pointer, resource)
            bset = 0
            for i in range(len(g.nodes) - 1, -1, -1):
                n = g.nodes[i]
                ln = lane_of[i]
                s, ws = S[ln], WS[ln]
                acc = 1 if n.x in written else 0
                if n.kind == "conv":
                    u = unit_of[n.idx]
                    if u.first is not n:
                        continue        # a group runs at its first member: every member's dy is final then
                    d = self._conv_desc(u, B)
                    keep.append(d)
                    M = B * u.ho * u.wo
                    uid = u.first.idx
                    raw = self.raw_unit[uid].data_ptr()
                    draw = self.draw_lane[ln].data_ptr()
                    dkey = ("draw", ln)
                    wl = ln
                    if stem_split and i < stem_end and ln == 0:   # filter gradient on lane 1
                        if sbuf:
                            draw, dkey = self.draw_stem2.data_ptr(), ("draw2", 0)
                        sbuf ^= 1
                        wl = 1
                    if uid in in_batch and uid not in batch_draw:   # the block's batched BN backward
                        grp = self.bn_batch[in_batch[uid][0]]
                        layers = (_ffi.BnBwdLayer * len(grp))()
                        reads, writes = [("r", v.first.idx) for v in grp] + [("p",)], [("ws", ln)]
                        for k, v in enumerate(grp):
                            vid = v.first.idx
                            ptr = self.drawb[bset][k].data_ptr()
                            batch_draw[vid] = (ptr, ("drawb", bset, k))
                            segs = [_ffi.BnSeg(D(m.y.buf), m.y.c_off, g.bufs[m.y.buf].c, m.cout,
                                               self._p(f"batch_normalization_{m.idx + 1}/beta"),
                                               self._gp(f"batch_normalization_{m.idx + 1}/beta")) for m in v.members]
                            layers[k].nseg = len(segs)
                            for j, sgm in enumerate(segs):
                                layers[k].segs[j] = sgm
                            layers[k].x = self.raw_unit[vid].data_ptr()
                            layers[k].x_c_off, layers[k].x_c_stride = 0, v.cout
                            layers[k].m, layers[k].c = B * v.ho * v.wo, v.cout
                            layers[k].mean = self.mean_unit[vid].data_ptr()
                            layers[k].invstd = self.invstd_unit[vid].data_ptr()
                            layers[k].dx = ptr
                            reads += [("d", m.y.buf, m.y.c_off) for m in v.members]
                            writes += [("drawb", bset, k), ("g", vid)]
                        keep.append(layers)
                        add(bwd, L.jr_bn_relu_bwd_batch, (dt, len(grp), ctypes.byref(layers), ws, wsb, s),
                            "bn_relu_bwd", ln, reads, writes,
                            nbytes=sum(3 * B * v.ho * v.wo * v.cout * self.esz for v in grp))
                        bset ^= 1
                    if uid in batch_draw:
                        draw, dkey = batch_draw[uid]
                    # one backward launch set for all members of the launch (segments:
                    # each member's upstream gradient slice, beta and dbeta)
                    pool_i = next((j for j, b in pool_bwd.items() if b == u.first.y.buf), None)
                    if pool_i is not None:    # the max-pool backward adds the BN reduce's sums
                        pn, m0 = g.nodes[pool_i], u.first
                        pd = self._pool_desc(pn, B)
                        keep.append(pd)
                        pargs = (dt, ctypes.byref(pd), self.argmax[pool_i].data_ptr(), D(pn.y.buf), D(pn.x), raw,
                                 u.cout, self.mean_unit[uid].data_ptr(), self.invstd_unit[uid].data_ptr(),
                                 self._p(f"batch_normalization_{m0.idx + 1}/beta"), draw,
                                 self._gp(f"batch_normalization_{m0.idx + 1}/beta"), ws, wsb)
                        pfn = L.jr_bn_relu_bwd_maxpool
                        if self.x6h:    # also the raw-output gradient's magnitude (dy_absmax of its GEMMs)
                            pfn, pargs = L.jr_bn_relu_bwd_maxpool_absmax, pargs + (self._dmax(u),)
                        add(bwd, pfn, pargs + (s,),
                            "bn_relu_bwd", ln, [("d", pn.y.buf, pn.y.c_off), ("am", pool_i), ("r", uid), ("p",)],
                            d_all(pn.x) + [dkey, ("g", uid), ("ws", ln)] + ([("dmax", uid)] if self.x6h else []),
                            nbytes=4 * M * u.cout * self.esz)
                    for grp in ([] if pool_i is not None or uid in batch_draw else self._bn_groups(u)):
                        co0 = grp[0][1]
                        cg = sum(m.cout for m, _ in grp)
                        segs = (_ffi.BnSeg * len(grp))(*[
                            _ffi.BnSeg(D(m.y.buf), m.y.c_off, g.bufs[m.y.buf].c, m.cout,
                                       self._p(f"batch_normalization_{m.idx + 1}/beta"),
                                       self._gp(f"batch_normalization_{m.idx + 1}/beta")) for m, _ in grp])
                        keep.append(segs)
                        bargs = (dt, len(grp), ctypes.byref(segs), raw, co0, u.cout, M, cg,
                                 self.mean_unit[uid].data_ptr() + 4 * co0, self.invstd_unit[uid].data_ptr() + 4 * co0,
                                 draw, ws, wsb)
                        bfn = L.jr_bn_relu_bwd_multi
                        if self.x6h:
                            bfn, bargs = L.jr_bn_relu_bwd_multi_absmax, bargs + (self._dmax(u),)
                        add(bwd, bfn, bargs + (s,),
                            "bn_relu_bwd", ln, [("d", m.y.buf, m.y.c_off) for m, _ in grp] + [("r", uid), ("p",)],
                            [dkey, ("g", uid), ("ws", ln)] + ([("dmax", uid)] if self.x6h else []),
                            nbytes=3 * M * cg * self.esz)
                    if x8p:             # the raw-output gradient as split planes (dgrad and wgrad operand)
                        drawp = self.drawp_lane[ln].data_ptr()
                        add(bwd, L.jr_split_x8p, (draw, M, u.cout, 0, u.cout, drawp, u.cout, 0, u.cout, M * u.cout, s),
                            "split_x8p", ln, [("draw", ln)], [("drawp", ln)], nbytes=10 * M * u.cout)
                        draw, dkey = drawp, ("drawp", ln)
                    def dgrad():
                        if u.x != g.input_buf:
                            add(bwd, L.jr_conv2d_bwd_data, (ctypes.byref(d), cdt, draw, self._wd(u), D(u.x), acc, ws,
                                                            wsb, s),
                                "conv_dgrad", ln, [dkey, wkey] + xw, d_all(u.x) + [("ws", ln)])
                            written.add(u.x)
                    if self.dgrad_first:
                        dgrad()
                    if uid in defer:
                        sg, _, nb = defer[uid]
                        add(bwd, L.jr_conv2d_bwd_filter_slabs, (ctypes.byref(d), cdt, AX(u.x), draw, sg.slabs, nb,
                                                                S[wl]),
                            "conv_wgrad", wl, ax_reads(u.x) + [dkey], [("slab", uid)])
                        pending.append((sg, uid))
                    elif wl != ln:
                        add(bwd, L.jr_conv2d_bwd_filter, (ctypes.byref(d), cdt, AX(u.x), draw,
                                                          self.grads.data_ptr() + 4 * u.koff,
                                                          ctypes.c_void_p(self.ws_stem.data_ptr()), wsb, S[wl]),
                            "conv_wgrad", wl, ax_reads(u.x) + [dkey], [("g", uid), ("wss",)])
                    else:
                        add(bwd, L.jr_conv2d_bwd_filter, (ctypes.byref(d), cdt, AX(u.x), draw,
                                                          self.grads.data_ptr() + 4 * u.koff, ws, wsb, s),
                            "conv_wgrad", ln, ax_reads(u.x) + [dkey], [("g", uid), ("ws", ln)])
                    if not self.dgrad_first:
                        dgrad()
                    trigger = False
                    while flush_at and flush_at[0] >= u.koff:
                        flush_at.pop(0)
                        trigger = True
                    if trigger:
                        flush()
                    bwd.append(Call("param_ready", u.koff, "hook", 0))
                elif n.kind == "maxpool" and i in pool_bwd:
                    continue            # with its producer's BN backward (jr_bn_relu_bwd_maxpool)
                elif n.kind == "maxpool":
                    d = self._pool_desc(n, B)
                    keep.append(d)
                    add(bwd, L.jr_maxpool3x3s2_bwd, (ctypes.byref(d), dt, self.argmax[i].data_ptr(), D(n.y.buf),
                                                     D(n.x), acc, s),
                        "maxpool_bwd", ln, [("am", i), ("d", n.y.buf, n.y.c_off)], d_all(n.x),
                        nbytes=B * n.c * (n.ho * n.wo * (self.esz + 1) + n.h * n.w * self.esz * (1 + acc)))
                    written.add(n.x)
                else:
                    d = self._pool_desc(n, B)
                    keep.append(d)
                    add(bwd, L.jr_avgpool3x3s1_bwd, (ctypes.byref(d), dt, D(n.y.buf), D(n.x), acc, s),
                        "avgpool_bwd", ln, [("d", n.y.buf, n.y.c_off)], d_all(n.x),
                        nbytes=B * n.c * (n.ho * n.wo + n.h * n.w * (1 + acc)) * self.esz)
                    written.add(n.x)
            flush()
            P, G = self.params.data_ptr(), self.grads.data_ptr()
            greads = [("g", u.first.idx) for u in self.cunits] + [("g", "dense")]
            if self.optimizer == "nesterov":
                add(opt, L.jr_nesterov_update, (P, G, self.accum.data_ptr(), self.nparam, self.lr,
                                                self.momentum, 1.0, s0), "nesterov", 0, greads, [("p",), ("acc",)],
                    nbytes=20 * self.nparam)
            elif self.optimizer == "momentum":
                add(opt, L.jr_momentum_update, (P, G, self.accum.data_ptr(), self.nparam, self.lr,
                                                self.momentum, 1.0, s0), "momentum", 0, greads, [("p",), ("acc",)])
            elif self.optimizer == "sgd":
                add(opt, L.jr_sgd_update, (P, G, self.nparam, self.lr, 1.0, s0), "sgd", 0, greads, [("p",)])
            else:   # adam: lr_t of the step is filled in by apply_update
                add(opt, L.jr_adam_update, (P, G, self.accum.data_ptr(), self.adam_v.data_ptr(), self.nparam,
                                            self.lr, self.adam_b1, self.adam_b2, self.adam_eps, 1.0, s0),
                    "adam", 0, greads, [("p",), ("acc",)])
        schedule(seq)
        self._calls[key] = (fwd, bwd, opt, keep, None)
        return self._calls[key]

    def _run(self, calls, events=None, hook: Optional[Callable[[int], None]] = None) -> None:
        for c in calls:
            if c.fn == "param_ready":
                # no join here: the hook fences the lanes onto ITS stream, and
                # only when a bucket is actually issued (fence_lanes); lane 0
                # never waits for lane 1 at a conv unit
                if hook is not None:
                    if self._join_each:     # round-5 behaviour, A/B runs only (JR_DP_JOIN_EACH=1)
                        self._join()
                    hook(c.args)
                continue
            st = self.lane_streams[c.lane]
            if self.precise_waits and not self._capturing:
                for lj, j in c.pwaits:      # the producing call on the other lane (jr.lanes.schedule)
                    ev = self._prod_ev.get(j)
                    if ev is None:          # producer never run in this process (e.g. backward() first): its tail
                        ev = self._tail_ev[lj]
                        ev.record(self.lane_streams[lj])
                        st.wait_event(ev)
                    elif self._native_ev:
                        _ffi.check("jr_stream_wait_event", self.lib.jr_stream_wait_event(self._lane_s[c.lane], ev))
                    else:
                        st.wait_event(ev)
            else:
                for lj in c.waits:          # the other lane's tail (jr.lanes.schedule)
                    ev = self._tail_ev[lj]
                    ev.record(self.lane_streams[lj])
                    st.wait_event(ev)
            rc = c.fn(*c.args)
            if rc:
                raise _ffi.JRError(c.name, rc, _ffi.last_error())
            if c.record and self.precise_waits and not self._capturing:
                ev = self._prod_ev.get(c.idx)
                if ev is None:
                    ev = self._prod_ev[c.idx] = self._new_event()
                if self._native_ev:
                    _ffi.check("jr_event_record", self.lib.jr_event_record(ev, self._lane_s[c.lane]))
                else:
                    ev.record(st)

    def _new_event(self):
        if not self._native_ev:
            return torch.cuda.Event()
        ev = ctypes.c_void_p()
        _ffi.check("jr_event_create", self.lib.jr_event_create(ctypes.byref(ev)))
        weakref.finalize(self, self.lib.jr_event_destroy, ev)
        return ev

    def _fork(self) -> None:
        """Every lane waits for the work enqueued on lane 0 so far."""
        if self.nlanes > 1:
            self._fork_ev.record(self.stream)
            for st in self.lane_streams[1:]:
                st.wait_event(self._fork_ev)

    def _join(self) -> None:
        """Lane 0 waits for every other lane's work enqueued so far."""
        for ev, st in zip(self._join_ev, self.lane_streams[1:]):
            ev.record(st)
            self.stream.wait_event(ev)

    def fence_lanes(self, stream) -> None:
        """`stream` (a consumer outside the lanes: the gradient all-reduce's
        stream) waits for the work enqueued on EVERY lane so far; the lanes
        themselves wait for nothing.  Used by jr.dist.BucketAllReduce at each
        bucket's issue point instead of joining the lanes onto lane 0."""
        if not hasattr(self, "_fence_ev"):
            self._fence_ev = [torch.cuda.Event() for _ in range(self.nlanes)]
        for ev, st in zip(self._fence_ev, self.lane_streams):
            ev.record(st)
            stream.wait_event(ev)

    # ------------------------------------------------------------------- data
    def set_batch(self, images, labels=None, n: Optional[int] = None) -> int:
        """Copy a batch (NHWC float32, or uint8 to be scaled by 1/255) into the
        input buffer.  Returns the batch size."""
        B = int(images.shape[0]) if n is None else n
        if B > self.batch:
            raise ValueError(f"batch {B} > planned {self.batch}")
        ib = self.g.bufs[self.g.input_buf]
        if tuple(images.shape[1:]) != (ib.h, ib.w, ib.c):
            raise ValueError(f"images must be [B,{ib.h},{ib.w},{ib.c}] NHWC, got {tuple(images.shape)}")
        with torch.cuda.stream(self.stream):
            x = torch.as_tensor(images)
            pixels = B * ib.h * ib.w
            if x.dtype == torch.uint8:
                xd = x.to(self.device, non_blocking=True).reshape(-1)
                _ffi.check("jr_image_u8_to_nhwc", self.lib.jr_image_u8_to_nhwc(
                    xd.data_ptr(), self.acts[self.g.input_buf].data_ptr(), self.dt, pixels, ib.c,
                    self.in_stride, self._s))
                self._keep_u8 = xd
            else:
                dst = self.acts[self.g.input_buf][:pixels * self.in_stride].view(pixels, self.in_stride)
                dst[:, ib.c:].zero_()
                dst[:, :ib.c].copy_(x.to(torch.float32).reshape(pixels, ib.c).to(self.device, non_blocking=True))
            if labels is not None:
                y = torch.as_tensor(labels, dtype=torch.float32).reshape(-1)
                if y.numel() != B * self.units:
                    raise ValueError("labels must have batch*units elements")
                self.labels[:y.numel()].copy_(y, non_blocking=True)
        return B

    # ------------------------------------------------------------------- runs
    def forward(self, B: Optional[int] = None) -> None:
        fwd, _, _, _, ev = self._build_calls(B or self.batch)
        self._fork()
        self._run(fwd, ev)
        self._join()

    def backward(self, B: Optional[int] = None, hook=None) -> None:
        _, bwd, _, _, ev = self._build_calls(B or self.batch)
        self._run(bwd, ev, hook)
        self._join()

    def apply_update(self, B: Optional[int] = None, grad_scale: float = 1.0) -> None:
        _, _, opt, _, ev = self._build_calls(B or self.batch)
        if grad_scale != 1.0 or self.optimizer == "adam":
            c = opt[0]
            args = list(c.args)
            args[-2] = grad_scale
            if self.optimizer == "adam":
                # TF ApplyAdam (training_ops.cc): alpha = lr * sqrt(1 - beta2_power)
                # / (1 - beta1_power), evaluated in the variable dtype (fp32,
                # left to right; np.sqrt of a float32 is correctly rounded like
                # Eigen's), from fp32 beta powers (so Adam steps run eagerly:
                # the scalar changes every step)
                f = np.float32
                self.adam_t += 1
                alpha = f(f(self.lr) * np.sqrt(f(1) - self.adam_b2p)) / (f(1) - self.adam_b1p)
                args[5] = float(f(alpha))
                self.adam_b1p = f(self.adam_b1p * f(self.adam_b1))
                self.adam_b2p = f(self.adam_b2p * f(self.adam_b2))
            opt = [dataclasses.replace(c, args=tuple(args))]
        self._run(opt, ev)

    def train_step(self, B: Optional[int] = None, allreduce=None) -> None:
        """fwd + bwd (+ bucketed all-reduce) + optimizer, enqueued on the lanes;
        everything is joined back onto self.stream before the optimizer."""
        B = B or self.batch
        if allreduce is None:
            self.forward(B)
            self.backward(B)
            self.apply_update(B)
            return
        self.forward(B)
        allreduce.begin(self)
        self.backward(B, hook=allreduce.param_ready)
        scale = allreduce.finish(self)
        self.apply_update(B, grad_scale=scale)

    def capture(self, B: Optional[int] = None) -> None:
        """Capture fwd+bwd+update for batch B into a HIP graph (single GPU;
        not for Adam, whose step scalar changes every step); the two lane
        streams are captured (fork/join by events) and become parallel
        branches of the graph.  At most two lanes: on ROCm 7.2, cross-waits
        among three or more captured streams crashed hipGraphInstantiate, and
        the same DAG built explicitly on one capturing stream (stream capture
        dependencies set per call) crashed hipGraphLaunch depending on the
        process's history; more lanes run eagerly."""
        B = B or self.batch
        if self.optimizer == "adam":
            raise ValueError("Adam steps run eagerly (the step's alpha is a host scalar)")
        if self.nlanes > 2:
            raise ValueError("HIP graph capture supports at most two lanes (more lanes run eagerly)")
        fwd, bwd, opt, _, _ = self._build_calls(B)
        torch.cuda.synchronize(self.device)
        _ffi.check("jr_graph_begin", self.lib.jr_graph_begin(self._s))
        # the producer waits become the graph's edges (two lanes at most: with
        # three, waits on events recorded mid-stream crashed hipGraphInstantiate
        # on ROCm 7.2); JR_GRAPH_PRECISE=0: tail waits (bf16 replay 10.04 vs
        # 9.28 ms per step, eager 9.31: profiles/r05_graph_probe.txt)
        self._capturing = os.environ.get("JR_GRAPH_PRECISE", "1") == "0"
        try:
            self._fork()
            self._run(fwd)
            self._join()
            self._run(bwd)
            self._join()
            self._run(opt)
        finally:
            self._capturing = False
            ex = ctypes.c_void_p()
            _ffi.check("jr_graph_end", self.lib.jr_graph_end(self._s, ctypes.byref(ex)))
        self._graphs[B] = ex.value

    def replay(self, B: Optional[int] = None) -> None:
        B = B or self.batch
        _ffi.check("jr_graph_launch", self.lib.jr_graph_launch(ctypes.c_void_p(self._graphs[B]), self._s))

    def synchronize(self) -> None:
        """Wait for every lane, then jr_device_check: a device-side failure
        of any launch since the last check (a stream-K hand-off count word not
        left zero) raises JRError here instead of leaving wrong numbers."""
        for st in self.lane_streams:
            st.synchronize()
        _ffi.device_check()

    def loss_value(self) -> float:
        self.synchronize()
        return float(self.loss[0].item())

    def predictions(self, B: Optional[int] = None) -> np.ndarray:
        B = B or self.batch
        self.synchronize()
        return self.probs[:B * self.units].cpu().numpy().reshape(B, self.units)

    def close(self) -> None:
        """Destroy this engine's HIP graph executables (also on collection)."""
        graphs = getattr(self, "_graphs", None)
        if not graphs:
            return
        for ex in graphs.values():
            self.lib.jr_graph_destroy(ctypes.c_void_p(ex))
        graphs.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:   # interpreter shutdown: the library may be gone
            pass
