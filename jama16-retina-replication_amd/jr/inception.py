"""Inception-v3 graph as an explicit op list (no tracing).

Topology, layer order and parameter order follow the Keras InceptionV3 that
the reference instantiates at train.py:129-130
(`tf.keras.applications.InceptionV3(include_top=False, pooling='avg')`,
keras_applications/inception_v3.py [TF-3P]) followed by the dense head of
train.py:133.  SURVEY.md Appendix A lists the same table.

Every Conv2D(use_bias=False) -> BatchNormalization(scale=False) -> ReLU
("conv2d_bn") is one ConvNode.  Concatenations do not exist as ops: each
branch's final node writes its channel slice of the block's output buffer
(concat-free writes), so a block output is one NHWC buffer.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Tuple

BN_EPS = 1e-3  # Keras BatchNormalization default epsilon (conv2d_bn uses it)


@dataclass
class Buf:
    id: int
    name: str
    h: int
    w: int
    c: int


@dataclass
class TRef:
    """Channel slice [c_off, c_off + c) of buffer `buf`."""
    buf: int
    c_off: int
    c: int


@dataclass
class ConvNode:
    idx: int              # 0-based Keras creation index (conv2d_{idx+1})
    x: int                # input buffer id (always a whole buffer)
    y: TRef               # output slice (after BN + ReLU)
    cin: int
    cout: int
    kh: int
    kw: int
    stride: int
    padding: str          # 'same' | 'valid'
    h: int
    w: int
    ho: int
    wo: int
    kind: str = "conv"

    @property
    def pad_h(self) -> int:
        return (self.kh - 1) // 2 if self.padding == "same" else 0

    @property
    def pad_w(self) -> int:
        return (self.kw - 1) // 2 if self.padding == "same" else 0

    @property
    def name(self) -> str:
        return f"conv2d_{self.idx + 1}"

    def macs_per_image(self) -> int:
        return self.ho * self.wo * self.cout * self.kh * self.kw * self.cin


@dataclass
class PoolNode:
    kind: str             # 'maxpool' (3x3/2 valid) | 'avgpool' (3x3/1 same, exclude pad)
    x: int
    y: TRef
    h: int
    w: int
    ho: int
    wo: int
    c: int


@dataclass
class Graph:
    height: int
    width: int
    units: int
    bufs: List[Buf] = field(default_factory=list)
    nodes: list = field(default_factory=list)
    input_buf: int = 0
    output_buf: int = -1          # mixed10
    params: List[Tuple[str, Tuple[int, ...]]] = field(default_factory=list)

    @property
    def convs(self) -> List[ConvNode]:
        return [n for n in self.nodes if n.kind == "conv"]

    def num_params(self) -> int:
        total = 0
        for _, shp in self.params:
            k = 1
            for s in shp:
                k *= s
            total += k
        return total

    def macs_per_image(self) -> int:
        return sum(n.macs_per_image() for n in self.convs)

    def train_flops_per_image(self) -> int:
        """fwd + dgrad + wgrad conv FLOPs (2 per MAC); conv1 has no dgrad."""
        f = 0
        for n in self.convs:
            m = n.macs_per_image()
            f += 2 * m * (2 if n.idx == 0 else 3)
        return f

    def bn_elems_per_image(self) -> int:
        return sum(n.ho * n.wo * n.cout for n in self.convs)


def _out(h: int, k: int, s: int, padding: str) -> int:
    if padding == "same":
        return (h + s - 1) // s
    return (h - k) // s + 1


class _Builder:
    def __init__(self, g: Graph):
        self.g = g
        self.nconv = 0

    def buf(self, name: str, h: int, w: int, c: int) -> int:
        b = Buf(len(self.g.bufs), name, h, w, c)
        self.g.bufs.append(b)
        return b.id

    def conv(self, x: int, cout: int, kh: int, kw: int, stride: int = 1, padding: str = "same",
             out: TRef | None = None, name: str | None = None) -> TRef:
        xb = self.g.bufs[x]
        if padding == "same":
            assert stride == 1, "Inception-v3 has no strided 'same' conv"
        ho, wo = _out(xb.h, kh, stride, padding), _out(xb.w, kw, stride, padding)
        if out is None:
            out = TRef(self.buf(name or f"conv2d_{self.nconv + 1}", ho, wo, cout), 0, cout)
        ob = self.g.bufs[out.buf]
        assert (ob.h, ob.w) == (ho, wo) and out.c == cout and out.c_off + cout <= ob.c
        node = ConvNode(self.nconv, x, out, xb.c, cout, kh, kw, stride, padding, xb.h, xb.w, ho, wo)
        self.g.nodes.append(node)
        self.g.params.append((f"{node.name}/kernel", (kh, kw, xb.c, cout)))
        self.g.params.append((f"batch_normalization_{self.nconv + 1}/beta", (cout,)))
        self.nconv += 1
        return out

    def pool(self, kind: str, x: int, out: TRef | None = None, name: str = "pool") -> TRef:
        xb = self.g.bufs[x]
        if kind == "maxpool":
            ho, wo = _out(xb.h, 3, 2, "valid"), _out(xb.w, 3, 2, "valid")
        else:
            ho, wo = xb.h, xb.w
        if out is None:
            out = TRef(self.buf(name, ho, wo, xb.c), 0, xb.c)
        ob = self.g.bufs[out.buf]
        assert (ob.h, ob.w) == (ho, wo) and out.c == xb.c
        self.g.nodes.append(PoolNode(kind, x, out, xb.h, xb.w, ho, wo, xb.c))
        return out


def build_inception_v3(height: int = 299, width: int = 299, units: int = 1) -> Graph:
    """Keras InceptionV3(include_top=False, pooling='avg') + Dense(units)."""
    g = Graph(height, width, units)
    b = _Builder(g)
    x = b.buf("input", height, width, 3)
    g.input_buf = x

    # stem (keras_applications inception_v3: conv2d_bn x3, maxpool, conv2d_bn x2, maxpool)
    t = b.conv(x, 32, 3, 3, 2, "valid")
    t = b.conv(t.buf, 32, 3, 3, 1, "valid")
    t = b.conv(t.buf, 64, 3, 3)
    t = b.pool("maxpool", t.buf, name="max_pooling2d_1")
    t = b.conv(t.buf, 80, 1, 1, 1, "valid")
    t = b.conv(t.buf, 192, 3, 3, 1, "valid")
    t = b.pool("maxpool", t.buf, name="max_pooling2d_2")
    x = t.buf

    # mixed0..2: 35x35 -> 256 / 288 / 288
    for i, pool_c in enumerate((32, 64, 64)):
        xb = g.bufs[x]
        tot = 64 + 64 + 96 + pool_c
        o = b.buf(f"mixed{i}", xb.h, xb.w, tot)
        b.conv(x, 64, 1, 1, out=TRef(o, 0, 64))
        t = b.conv(x, 48, 1, 1)
        b.conv(t.buf, 64, 5, 5, out=TRef(o, 64, 64))
        t = b.conv(x, 64, 1, 1)
        t = b.conv(t.buf, 96, 3, 3)
        b.conv(t.buf, 96, 3, 3, out=TRef(o, 128, 96))
        t = b.pool("avgpool", x, name=f"average_pooling2d_{i + 1}")
        b.conv(t.buf, pool_c, 1, 1, out=TRef(o, 224, pool_c))
        x = o

    # mixed3: 35 -> 17, 768
    xb = g.bufs[x]
    h3 = _out(xb.h, 3, 2, "valid")
    o = b.buf("mixed3", h3, _out(xb.w, 3, 2, "valid"), 384 + 96 + xb.c)
    b.conv(x, 384, 3, 3, 2, "valid", out=TRef(o, 0, 384))
    t = b.conv(x, 64, 1, 1)
    t = b.conv(t.buf, 96, 3, 3)
    b.conv(t.buf, 96, 3, 3, 2, "valid", out=TRef(o, 384, 96))
    b.pool("maxpool", x, out=TRef(o, 480, xb.c))
    x = o

    # mixed4..7: 17x17x768
    for i, c7 in enumerate((128, 160, 160, 192)):
        xb = g.bufs[x]
        o = b.buf(f"mixed{4 + i}", xb.h, xb.w, 768)
        b.conv(x, 192, 1, 1, out=TRef(o, 0, 192))
        t = b.conv(x, c7, 1, 1)
        t = b.conv(t.buf, c7, 1, 7)
        b.conv(t.buf, 192, 7, 1, out=TRef(o, 192, 192))
        t = b.conv(x, c7, 1, 1)
        t = b.conv(t.buf, c7, 7, 1)
        t = b.conv(t.buf, c7, 1, 7)
        t = b.conv(t.buf, c7, 7, 1)
        b.conv(t.buf, 192, 1, 7, out=TRef(o, 384, 192))
        t = b.pool("avgpool", x, name=f"average_pooling2d_{4 + i}")
        b.conv(t.buf, 192, 1, 1, out=TRef(o, 576, 192))
        x = o

    # mixed8: 17 -> 8, 1280
    xb = g.bufs[x]
    o = b.buf("mixed8", _out(xb.h, 3, 2, "valid"), _out(xb.w, 3, 2, "valid"), 320 + 192 + xb.c)
    t = b.conv(x, 192, 1, 1)
    b.conv(t.buf, 320, 3, 3, 2, "valid", out=TRef(o, 0, 320))
    t = b.conv(x, 192, 1, 1)
    t = b.conv(t.buf, 192, 1, 7)
    t = b.conv(t.buf, 192, 7, 1)
    b.conv(t.buf, 192, 3, 3, 2, "valid", out=TRef(o, 320, 192))
    b.pool("maxpool", x, out=TRef(o, 512, xb.c))
    x = o

    # mixed9, mixed10: 8x8x2048 (mixed9_{i} and the unnamed inner concat are
    # flattened into the block buffer)
    for i in range(2):
        xb = g.bufs[x]
        o = b.buf(f"mixed{9 + i}", xb.h, xb.w, 2048)
        b.conv(x, 320, 1, 1, out=TRef(o, 0, 320))
        t = b.conv(x, 384, 1, 1)
        b.conv(t.buf, 384, 1, 3, out=TRef(o, 320, 384))
        b.conv(t.buf, 384, 3, 1, out=TRef(o, 704, 384))
        t = b.conv(x, 448, 1, 1)
        t = b.conv(t.buf, 384, 3, 3)
        b.conv(t.buf, 384, 1, 3, out=TRef(o, 1088, 384))
        b.conv(t.buf, 384, 3, 1, out=TRef(o, 1472, 384))
        t = b.pool("avgpool", x, name=f"average_pooling2d_{8 + i}")
        b.conv(t.buf, 192, 1, 1, out=TRef(o, 1856, 192))
        x = o

    g.output_buf = x
    feat_c = g.bufs[x].c
    g.params.append(("dense/kernel", (feat_c, units)))
    g.params.append(("dense/bias", (units,)))
    assert b.nconv == 94
    return g
