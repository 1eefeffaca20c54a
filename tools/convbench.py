"""Diagnostic: time conv fwd GEMMs (no split-K) per tile config in normal /
no-MFMA / no-DMA / no-LDS-read variants to see which side bounds the kernel.
  python tools/convbench.py [cfg,cfg,...] [x8]"""
import ctypes, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jama16-retina-replication_amd"))
import torch
from jr import _ffi
_ffi.init(0)
L = _ffi.load()
L.jr_conv2d_debug_time.restype = ctypes.c_int
L.jr_conv2d_debug_time.argtypes = [ctypes.POINTER(_ffi.ConvDesc), ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_float),
                                   ctypes.c_void_p]
cases = {"conv5 73x73 80->192 3x3": (64, 73, 73, 80, 192, 3, 3, 1, 0),
         "mixed 35x35 288->64 1x1": (64, 35, 35, 288, 64, 1, 1, 1, 0),
         "gemm-like 17x17 768->192 1x1": (64, 17, 17, 768, 192, 1, 1, 1, 0),
         "mixed10 8x8 448->384 3x3": (64, 8, 8, 448, 384, 3, 3, 1, 1)}
CFGS = [int(c) for c in sys.argv[1].split(",")] if len(sys.argv) > 1 and sys.argv[1] else [0, 2, 3, 11, 13]
X8 = len(sys.argv) > 2 and sys.argv[2] == "x8"     # JR_F32_X8 kernel; variant 4 = no operand split
VARIANTS = (16, 17, 18, 19, 20) if X8 else (0, 1, 2, 3)
for name, (n, h, w, ci, co, kh, kw, s, p) in cases.items():
    ho, wo = (h + 2 * p - kh) // s + 1, (w + 2 * p - kw) // s + 1
    d = _ffi.ConvDesc(n, h, w, ci, co, kh, kw, s, s, p, p, ho, wo, 0, ci, 0, co)
    x = torch.randn(n * h * w * ci, device="cuda")
    wt = torch.randn(kh * kw * ci * co, device="cuda") * 0.05
    y = torch.zeros(n * ho * wo * co, device="cuda")
    flops = 2.0 * n * ho * wo * co * kh * kw * ci
    for cfg in CFGS:
        res = []
        for dbg in VARIANTS:
            ms = ctypes.c_float()
            rc = L.jr_conv2d_debug_time(ctypes.byref(d), cfg, dbg, x.data_ptr(), wt.data_ptr(), y.data_ptr(), 2,
                                        ctypes.byref(ms), None)
            if rc:
                res.append(f"dbg{dbg}: n/a")
                continue
            L.jr_conv2d_debug_time(ctypes.byref(d), cfg, dbg, x.data_ptr(), wt.data_ptr(), y.data_ptr(), 10, ctypes.byref(ms), None)
            t = ms.value / 10
            res.append(f"dbg{dbg}: {t*1e3:8.1f}us {flops/t/1e9:6.1f}TF")
        print(f"{name:32s} cfg{cfg}: " + " | ".join(res), flush=True)
