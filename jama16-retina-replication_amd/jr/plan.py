"""Launch plan of the conv layers and the engine's internal parameter layout.

Sibling fusion: in every Inception block several 1x1 'same' conv2d_bn
layers read the SAME input buffer (mixed0-2: the 64 / 48 / 64 branch heads,
mixed4-7: 192 / c7 / c7, mixed8: 192 / 192, mixed9-10: 320 / 384 / 448; see
SURVEY.md App. A).  They are one GEMM with N = sum of their c_out: the
engine stores their kernels side by side as one [c_in][sum c_out] block, so
one implicit-GEMM launch computes all of them forward, one writes all their
filter gradients, and one computes their summed data gradient (instead of
one accumulate-into-dx launch per layer).  Each member keeps its own
BatchNormalization (per-channel, so the group's statistics are the members'
statistics), its own beta and its own output slice.  The arithmetic per
output element is unchanged: each output channel is still the dot product of
the same input pixel with the same kernel column.

Internal layout: the flat fp32 parameter buffer holds the tensors in Keras
creation order (jr.init.param_layout), except that a fused group's kernel
block and all its members' betas sit together at the position of the group's
first kernel.  Backward visits the layers in reverse order, so every byte at
offsets >= the offset of the layer just finished is final — the invariant
the bucketed all-reduce (jr.dist) relies on — and the group's parameters
all become final at once, when the group's backward runs.  Checkpoints,
params_numpy() and grads_numpy() use the Keras layout; to_internal /
to_keras convert.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Tuple

import numpy as np

from .inception import ConvNode, Graph
from .init import ALIGN, param_layout


@dataclass
class ConvUnit:
    """One implicit-GEMM conv launch: one conv2d_bn layer or a fused group."""
    members: List[ConvNode]
    col_off: List[int]
    koff: int = 0                     # internal offset of the kernel block

    @property
    def first(self) -> ConvNode:
        return self.members[0]

    @property
    def fused(self) -> bool:
        return len(self.members) > 1

    @property
    def cout(self) -> int:
        return sum(n.cout for n in self.members)

    @property
    def name(self) -> str:
        if not self.fused:
            return self.first.name
        return "conv2d_" + "+".join(str(n.idx + 1) for n in self.members)

    def __getattr__(self, k):          # geometry shared by all members
        if k in ("x", "cin", "kh", "kw", "stride", "padding", "h", "w", "ho", "wo", "pad_h", "pad_w"):
            return getattr(self.members[0], k)
        raise AttributeError(k)

    def macs_per_image(self) -> int:
        return sum(n.macs_per_image() for n in self.members)


@dataclass
class Plan:
    units: List[ConvUnit]
    unit_of: Dict[int, ConvUnit]                  # conv idx -> unit
    layout: List[Tuple[str, tuple, int, int]]     # internal (name, shape, off, size)
    nparam: int
    poff: Dict[str, int]                          # contiguous tensors: betas, dense, unfused kernels
    kview: Dict[str, Tuple[int, int, int, int, int]] = field(default_factory=dict)
    # conv kernel name -> (block offset, row stride, column offset, rows, cols)

    def to_internal(self, g: Graph, flat: np.ndarray) -> np.ndarray:
        keras, total = param_layout(g.params)
        flat = np.asarray(flat, np.float32)
        if flat.size != total:
            raise ValueError(f"expected {total} parameters (Keras layout), got {flat.size}")
        out = np.zeros(self.nparam, np.float32)
        for name, shape, off, size in keras:
            src = flat[off:off + size]
            if name in self.kview:
                o, ld, co, rows, cols = self.kview[name]
                out[o:o + rows * ld].reshape(rows, ld)[:, co:co + cols] = src.reshape(rows, cols)
            else:
                o = self.poff[name]
                out[o:o + size] = src
        return out

    def to_keras(self, g: Graph, flat: np.ndarray) -> np.ndarray:
        keras, total = param_layout(g.params)
        flat = np.asarray(flat, np.float32)
        out = np.zeros(total, np.float32)
        for name, shape, off, size in keras:
            if name in self.kview:
                o, ld, co, rows, cols = self.kview[name]
                out[off:off + size] = flat[o:o + rows * ld].reshape(rows, ld)[:, co:co + cols].ravel()
            else:
                o = self.poff[name]
                out[off:off + size] = flat[o:o + size]
        return out


def sibling_groups(g: Graph) -> List[List[ConvNode]]:
    """1x1 stride-1 conv2d_bn layers reading the same buffer, >= 2 of them."""
    by_input: Dict[int, List[ConvNode]] = {}
    for n in g.convs:
        if n.kh == 1 and n.kw == 1 and n.stride == 1:
            by_input.setdefault(n.x, []).append(n)
    return [v for v in by_input.values() if len(v) > 1]


def build_plan(g: Graph, fuse_siblings: bool = True) -> Plan:
    groups = sibling_groups(g) if fuse_siblings else []
    unit_of: Dict[int, ConvUnit] = {}
    for mem in groups:
        offs, c = [], 0
        for n in mem:
            offs.append(c)
            c += n.cout
        u = ConvUnit(list(mem), offs)
        for n in mem:
            unit_of[n.idx] = u
    units = []
    for n in g.convs:
        if n.idx not in unit_of:
            unit_of[n.idx] = ConvUnit([n], [0])
        u = unit_of[n.idx]
        if u.first is n:
            units.append(u)

    shapes = dict(g.params)
    layout, poff, kview = [], {}, {}
    off = 0

    def alloc(name, shape, size):
        nonlocal off
        layout.append((name, tuple(shape), off, size))
        o = off
        off += (size + ALIGN - 1) // ALIGN * ALIGN
        return o

    conv_by_name = {n.name: n for n in g.convs}
    done = set()
    for name, shape in g.params:
        if name in done:
            continue
        base = name.split("/")[0]
        n = conv_by_name.get(base)
        if n is not None and unit_of[n.idx].fused:
            u = unit_of[n.idx]
            rows = n.kh * n.kw * n.cin
            u.koff = alloc(u.name + "/kernel", (n.kh, n.kw, n.cin, u.cout), rows * u.cout)
            for m, co in zip(u.members, u.col_off):
                kview[f"{m.name}/kernel"] = (u.koff, u.cout, co, rows, m.cout)
                done.add(f"{m.name}/kernel")
            for m in u.members:
                bname = f"batch_normalization_{m.idx + 1}/beta"
                poff[bname] = alloc(bname, shapes[bname], m.cout)
                done.add(bname)
            continue
        size = int(np.prod(shape))
        o = alloc(name, shape, size)
        poff[name] = o
        if n is not None and name.endswith("/kernel"):
            unit_of[n.idx].koff = o
    return Plan(units, unit_of, layout, off, poff, kview)
