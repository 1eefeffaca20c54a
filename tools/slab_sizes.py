"""Filter-gradient split-K slab bytes per layer of the 299^2 B=64 plan (pinned
tiles), fp32 (x8) and bf16: what a deferred jr_wgrad_reduce would read.
python tools/slab_sizes.py   (GPU box: the Engine allocates on cuda:0)"""
import sys
sys.path.insert(0, "jama16-retina-replication_amd")
import ctypes
from jr.engine import Engine
from jr import _ffi
for dt in ("f32", "bf16"):
    e = Engine(64, 299, 299, dtype=dt, seed=0)
    L = e.lib
    sizes = []
    for u in e.cunits:
        d = e._conv_desc(u, 64)
        sg = _ffi.WgradSeg()
        _ffi.check("seg", L.jr_conv2d_wgrad_seg(ctypes.byref(d), e.cdt, ctypes.byref(sg)))
        if sg.splits > 1:
            sizes.append((4 * sg.splits * sg.m * sg.n / 2**20, sg.splits, sg.m * sg.n, u.first.name if hasattr(u.first, "name") else u.first.idx))
    sizes.sort(reverse=True)
    print(dt, len(sizes), "split layers, total %.0f MB" % sum(s[0] for s in sizes))
    for s in sizes[:12]:
        print("  %.1f MB splits %d params %d %s" % s)
    import numpy as np
    a = np.array([s[0] for s in sizes])
    for t in (2, 4, 8, 16, 32, 64):
        print("  <= %d MB: %d layers, %.0f MB" % (t, (a <= t).sum(), a[a <= t].sum()))
