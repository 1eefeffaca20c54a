"""A trial tile-table file (for JR_TILE_TABLES A/B runs): the pinned MI355X
tables with every split-K filter-gradient GEMM of the 299^2 B=64 training
tables replaced by the stream-K grid of the same tile -- no split-K slabs, so
no deferred jr_wgrad_reduce for those layers -- where
the filter gradient has at least `min_out` elements (a GEMM of few output
tiles cuts each into hundreds of stream-K pieces that one block sums).
python tools/sk_wgrad_tables.py <out.json> [min_out]"""
import copy
import ctypes
import json
import os
import sys
import types

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jama16-retina-replication_amd"))
from jr import _ffi, inception, plan as P  # noqa: E402
from jr.engine import Engine  # noqa: E402

out = sys.argv[1]
min_out = int(sys.argv[2]) if len(sys.argv) > 2 else 100000   # filter-gradient elements (M x N) at least
L = _ffi.load()
src = os.path.join(os.path.dirname(__file__), "..", "jama16-retina-replication_amd", "jr", "tiles_mi355x.json")
doc = json.load(open(src))
SK = {"x8": (2, 28, 14), "bf16": (1, 33, 17)}      # dtype code, first stream-K id, standard tiles
changed = 0
for t in doc["tables"]:
    if not (t["train"] and t["batch"] == 64 and t["height"] == 299 and t["conv_math"] in SK):
        continue
    code, sk0, nstd = SK[t["conv_math"]]
    g = inception.build_inception_v3(299, 299)
    pl = P.build_plan(g)
    fake = types.SimpleNamespace(x8p=False, in_stride=(4 if t["conv_math"] == "x8" else 8), g=g)
    for u in pl.units:
        d = Engine._conv_desc(fake, u, 64)
        f, wg, dg = t["configs"][u.name]
        tile = wg & 255
        if wg < 0 or tile >= nstd:
            continue
        L.jr_conv2d_set_config(ctypes.byref(d), _ffi.JR_CONV_BWD_FILTER, code, 0, wg)
        sg = _ffi.WgradSeg()
        _ffi.check("seg", L.jr_conv2d_wgrad_seg(ctypes.byref(d), code, ctypes.byref(sg)))
        L.jr_conv2d_set_config(ctypes.byref(d), _ffi.JR_CONV_BWD_FILTER, code, 0, -1)
        if sg.splits > 1 and sg.m * sg.n >= min_out:
            t["configs"][u.name] = [f, sk0 + tile, dg]
            changed += 1
            print(f"{t['conv_math']:5s} {u.name:26s} wgrad {wg} -> {sk0 + tile} (split-K {sg.splits} slabs of "
                  f"{sg.m}x{sg.n})")
json.dump(doc, open(out, "w"), indent=0)
print("changed", changed)
