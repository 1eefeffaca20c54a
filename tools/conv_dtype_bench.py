"""Per-layer conv timing across conv dtypes (autotuned, public C-ABI calls):
JR_F32_X8 (in-register split), JR_F32_X8P (pre-split planes), JR_BF16, and
optionally JR_F32.  B = 64 at 299^2 geometry.

  python tools/conv_dtype_bench.py [dtypes, default 2,3,1]
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jama16-retina-replication_amd"))
import torch  # noqa: E402
from jr import _ffi  # noqa: E402

_ffi.init(0)
L = _ffi.load()
NAMES = {0: "f32", 1: "bf16", 2: "x8", 3: "x8p"}
DTS = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [2, 3, 1]
cases = {"conv5 73x73 80->192 3x3": (64, 73, 73, 80, 192, 3, 3, 1, 0),
         "conv3 147x147 32->64 3x3 s": (64, 147, 147, 32, 64, 3, 3, 1, 1),
         "mixed 35x35 288->64 1x1": (64, 35, 35, 288, 64, 1, 1, 1, 0),
         "mixed 35x35 48->64 5x5": (64, 35, 35, 48, 64, 5, 5, 1, 2),
         "mixed3 35x35 288->384 3x3/2": (64, 35, 35, 288, 384, 3, 3, 2, 0),
         "17x17 768->512 1x1 (fused)": (64, 17, 17, 768, 512, 1, 1, 1, 0),
         "17x17 192->192 1x7": (64, 17, 17, 192, 192, 1, 7, 1, -1),
         "8x8 448->384 3x3": (64, 8, 8, 448, 384, 3, 3, 1, 1),
         "8x8 2048->1152 1x1 (fused)": (64, 8, 8, 2048, 1152, 1, 1, 1, 0)}


def timed(fn, reps=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


tot = {dt: 0.0 for dt in DTS}
for name, (n, h, w, ci, co, kh, kw, s, p) in cases.items():
    ph, pw = (0, 3) if p == -1 else (p, p)
    ho, wo = (h + 2 * ph - kh) // s + 1, (w + 2 * pw - kw) // s + 1
    d = _ffi.ConvDesc(n, h, w, ci, co, kh, kw, s, s, ph, pw, ho, wo, 0, ci, 0, co)
    macs = n * ho * wo * co * kh * kw * ci
    line = f"{name:30s}"
    for dt in DTS:
        pl = 3 if dt == 3 else 1
        esz = 2 if dt in (1, 3) else 4
        et = torch.bfloat16 if esz == 2 else torch.float32
        x = torch.randn(pl * n * h * w * ci, device="cuda").to(et)
        wt = (torch.randn(pl * kh * kw * ci * co, device="cuda") * 0.05).to(et)
        dy = torch.randn(pl * n * ho * wo * co, device="cuda").to(et)
        y = torch.zeros(n * ho * wo * co, device="cuda", dtype=torch.bfloat16 if dt == 1 else torch.float32)
        dx = torch.zeros(n * h * w * ci, device="cuda", dtype=torch.bfloat16 if dt == 1 else torch.float32)
        dw = torch.zeros(kh * kw * ci * co, device="cuda")
        wsb = max(L.jr_conv2d_workspace_size(ctypes.byref(d), op, dt) for op in range(3))
        ws = torch.zeros(wsb // 4 + 4, device="cuda")
        args = {0: (x, wt, y), 1: (dy, wt, dx), 2: (x, dy, dw)}
        for op in range(3):
            a, b, c = args[op]
            _ffi.check("tune", L.jr_conv2d_autotune(ctypes.byref(d), op, dt, a.data_ptr(), b.data_ptr(), c.data_ptr(),
                                                     ws.data_ptr(), wsb, None))
        us = [timed(lambda: _ffi.check("f", L.jr_conv2d_fwd(ctypes.byref(d), dt, x.data_ptr(), wt.data_ptr(),
                                                            y.data_ptr(), ws.data_ptr(), wsb, None))),
              timed(lambda: _ffi.check("d", L.jr_conv2d_bwd_data(ctypes.byref(d), dt, dy.data_ptr(), wt.data_ptr(),
                                                                 dx.data_ptr(), 0, ws.data_ptr(), wsb, None))),
              timed(lambda: _ffi.check("w", L.jr_conv2d_bwd_filter(ctypes.byref(d), dt, x.data_ptr(), dy.data_ptr(),
                                                                   dw.data_ptr(), ws.data_ptr(), wsb, None)))]
        tot[dt] += sum(us)
        line += f" | {NAMES[dt]:4s} " + " ".join(f"{u:7.1f}" for u in us) + f" ({3 * 2 * macs / sum(us) / 1e6:6.1f} TF)"
    print(line, flush=True)
print("total us: " + ", ".join(f"{NAMES[dt]} {tot[dt]:.0f}" for dt in DTS))
