"""Diagnostic: stream-K x8 GEMMs (ids 28..41) vs the split-K configs of the
committed x8 training table, per conv op of representative layers at B=64
(each timed over 20 back-to-back calls after warm-up; the split-K time
includes its reduce launch, as in the step).
  python tools/sk_probe.py"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jama16-retina-replication_amd"))
import torch  # noqa: E402
from jr import _ffi  # noqa: E402

_ffi.init(0)
L = _ffi.load()
X8 = _ffi.JR_F32_X8
LAYERS = {"17^2 1x7 192->192": (64, 17, 17, 192, 192, 1, 7, 1, 0, 3),
          "17^2 1x1 768->576": (64, 17, 17, 768, 576, 1, 1, 1, 0, 0),
          "35^2 3x3 96->96": (64, 35, 35, 96, 96, 3, 3, 1, 1, 1),
          "35^2 5x5 48->64": (64, 35, 35, 48, 64, 5, 5, 1, 2, 2),
          "8^2 3x3 448->384": (64, 8, 8, 448, 384, 3, 3, 1, 1, 1),
          "8^2 1x1 2048->1152": (64, 8, 8, 2048, 1152, 1, 1, 1, 0, 0),
          "73^2 3x3 80->192": (64, 73, 73, 80, 192, 3, 3, 1, 0, 0)}


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for name, (n, h, w, ci, co, kh, kw, s, ph, pw) in LAYERS.items():
    ho, wo = (h + 2 * ph - kh) // s + 1, (w + 2 * pw - kw) // s + 1
    d = _ffi.ConvDesc(n, h, w, ci, co, kh, kw, s, s, ph, pw, ho, wo, 0, ci, 0, co)
    flops = 2.0 * n * ho * wo * co * kh * kw * ci
    x = torch.randn(n * h * w * ci, device="cuda")
    wt = torch.randn(kh * kw * ci * co, device="cuda") * 0.05
    y = torch.zeros(n * ho * wo * co, device="cuda")
    dy = torch.randn(n * ho * wo * co, device="cuda")
    dx = torch.zeros(n * h * w * ci, device="cuda")
    dw = torch.zeros(kh * kw * ci * co, device="cuda")
    st = torch.zeros(2 * co, device="cuda")
    wsb = max(L.jr_conv2d_workspace_size(ctypes.byref(d), op, X8) for op in range(3))
    ws = torch.zeros(wsb // 4 + 4, device="cuda")
    ops = {0: lambda: L.jr_conv2d_fwd_bn_stats(ctypes.byref(d), X8, x.data_ptr(), wt.data_ptr(), y.data_ptr(), 1e-3,
                                               st.data_ptr(), st.data_ptr() + 4 * co, ws.data_ptr(), wsb, None),
           1: lambda: L.jr_conv2d_bwd_data(ctypes.byref(d), X8, dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), 0,
                                           ws.data_ptr(), wsb, None),
           2: lambda: L.jr_conv2d_bwd_filter(ctypes.byref(d), X8, x.data_ptr(), dy.data_ptr(), dw.data_ptr(),
                                             ws.data_ptr(), wsb, None)}
    for op, fn in ops.items():
        L.jr_conv2d_autotune(ctypes.byref(d), op, X8, *((x.data_ptr(), wt.data_ptr(), y.data_ptr()) if op == 0 else
                                                        (dy.data_ptr(), wt.data_ptr(), dx.data_ptr()) if op == 1 else
                                                        (x.data_ptr(), dy.data_ptr(), dw.data_ptr())),
                             ws.data_ptr(), wsb, None)
        best = L.jr_conv2d_get_config(ctypes.byref(d), op, X8, 0)
        tb = timed(fn)
        res = []
        for t in (11, 12, 13, 3, 1, 0, 4):
            L.jr_conv2d_set_config(ctypes.byref(d), op, X8, 0, 28 + t)
            res.append((timed(fn), t))
        L.jr_conv2d_set_config(ctypes.byref(d), op, X8, 0, -1)
        res.sort()
        print(f"{name:22s} op {op}: autotuned cfg {best & 255:2d}/{best >> 8:<3d} {tb:8.1f} us {flops / tb / 1e6:6.1f} TF/s"
              f" | stream-K best tile {res[0][1]:2d} {res[0][0]:8.1f} us {flops / res[0][0] / 1e6:6.1f} TF/s "
              f"({tb / res[0][0]:.2f}x)", flush=True)
