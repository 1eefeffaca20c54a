"""Diagnostic: is the x8 conv GEMM bound by power (operand bit activity)?
Times conv forward GEMMs (conv5 64 x 73^2 x 80 -> 192 3x3, a 17^2 1x7 and
a 35^2 1x1; tile `cfg`, one split) under JR_F32_X8 on (a) random fp32 operands, (b) operands that are
exactly bf16 (the m / l split terms are zero), (c) zeros -- ~1 s of
back-to-back launches each, then 50 timed.
  python tools/x8_power_probe.py [cfg]"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jama16-retina-replication_amd"))
import torch  # noqa: E402
from jr import _ffi  # noqa: E402

_ffi.init(0)
L = _ffi.load()
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 11
cases = {"conv5 73^2 80->192 3x3": (64, 73, 73, 80, 192, 3, 3, 0),
         "17^2 1x7 192->192": (64, 17, 17, 192, 192, 1, 7, 3),
         "35^2 1x1 288->64": (64, 35, 35, 288, 64, 1, 1, 0)}
for name, (n, h, w, ci, co, kh, kw, pw) in cases.items():
    ph = (kh - 1) // 2 if pw else 0
    ho, wo = h + 2 * ph - kh + 1, w + 2 * pw - kw + 1
    d = _ffi.ConvDesc(n, h, w, ci, co, kh, kw, 1, 1, ph, pw, ho, wo, 0, ci, 0, co)
    flops = 2.0 * n * ho * wo * co * kh * kw * ci
    for dt in (_ffi.JR_F32_X8,):
        _ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), 0, dt, 0, cfg | (1 << 8)))
    wsb = L.jr_conv2d_workspace_size(ctypes.byref(d), 0, _ffi.JR_F32_X8)
    ws = torch.zeros(wsb // 4 + 4, device="cuda")
    y = torch.zeros(n * ho * wo * co, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(1)
    xr = torch.randn(n * h * w * ci, device="cuda", generator=g)
    wr = torch.randn(kh * kw * ci * co, device="cuda", generator=g) * 0.05
    data = {"random": (xr, wr), "bf16-exact": (xr.bfloat16().float(), wr.bfloat16().float()),
            "zeros": (torch.zeros_like(xr), torch.zeros_like(wr))}
    for kind, (x, wt) in data.items():
        res = []
        for dt, wp in ((_ffi.JR_F32_X8, wt),):
            def run():
                _ffi.check("fwd", L.jr_conv2d_fwd(ctypes.byref(d), dt, x.data_ptr(), wp.data_ptr(), y.data_ptr(),
                                                  ws.data_ptr(), wsb, None))
            t0 = time.time()
            while time.time() - t0 < 1.0:
                for _ in range(20):
                    run()
                torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                run()
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / 50 / 1e3
            res.append(f"x8 {t * 1e6:7.1f} us {flops / t / 1e12:6.1f} TF/s")
        print(f"{name:24s} cfg {cfg:2d} {kind:10s}: " + " | ".join(res), flush=True)
    _ffi.check("reset", L.jr_conv2d_set_config(ctypes.byref(d), 0, _ffi.JR_F32_X8, 0, -1))
