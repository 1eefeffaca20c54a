"""Run one conv op repeatedly (for rocprofv3 --pmc passes and timing):
  python tools/conv_one.py <dtype 0|1|2|3> <op 0|1|2> <cfg|-1> [layer] [reps]
layers: conv5 (73^2 80->192 3x3, B=64), m17 (17^2 768->512 1x1), m8 (8^2 448->384 3x3),
        conv3, c17x7 (17^2 192->192 1x7 same), c35x3 (35^2 64->96 3x3 same)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jama16-retina-replication_amd"))
import torch  # noqa: E402
from jr import _ffi  # noqa: E402

LAYERS = {"conv5": (64, 73, 73, 80, 192, 3, 3, 1, 0), "m17": (64, 17, 17, 768, 512, 1, 1, 1, 0),
          "m8": (64, 8, 8, 448, 384, 3, 3, 1, 1), "conv3": (64, 147, 147, 32, 64, 3, 3, 1, 1),
          "c17x7": (64, 17, 17, 192, 192, 1, 7, 1, 0, 3), "c35x3": (64, 35, 35, 64, 96, 3, 3, 1, 1, 1)}
dt, op, cfg = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
layer = sys.argv[4] if len(sys.argv) > 4 else "conv5"
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 20
_ffi.init(0)
L = _ffi.load()
geo = LAYERS[layer]
n, h, w, ci, co, kh, kw, s = geo[:8]
ph, pw = geo[8:] if len(geo) == 10 else (geo[8], geo[8])
ho, wo = (h + 2 * ph - kh) // s + 1, (w + 2 * pw - kw) // s + 1
d = _ffi.ConvDesc(n, h, w, ci, co, kh, kw, s, s, ph, pw, ho, wo, 0, ci, 0, co)
pl = 3 if dt == 3 else 1
et = torch.bfloat16 if dt in (1, 3) else torch.float32
ot = torch.bfloat16 if dt == 1 else torch.float32
x = torch.randn(pl * n * h * w * ci, device="cuda").to(et)
wt = (torch.randn(pl * kh * kw * ci * co, device="cuda") * 0.05).to(et)
dy = torch.randn(pl * n * ho * wo * co, device="cuda").to(et)
y = torch.zeros(n * ho * wo * co, device="cuda", dtype=ot)
dx = torch.zeros(n * h * w * ci, device="cuda", dtype=ot)
dw = torch.zeros(kh * kw * ci * co, device="cuda")
wsb = max(L.jr_conv2d_workspace_size(ctypes.byref(d), o, dt) for o in range(3)) * 2
ws = torch.zeros(wsb // 4 + 4, device="cuda")
if cfg >= 0:
    for ph in range(s * s if op == 1 else 1):
        _ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), op, dt, ph, cfg))
print("cfg", L.jr_conv2d_get_config(ctypes.byref(d), op, dt, 0), flush=True)
if op == 0:
    fn = lambda: L.jr_conv2d_fwd(ctypes.byref(d), dt, x.data_ptr(), wt.data_ptr(), y.data_ptr(), ws.data_ptr(), wsb, None)  # noqa: E731
elif op == 1:
    fn = lambda: L.jr_conv2d_bwd_data(ctypes.byref(d), dt, dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), 0, ws.data_ptr(), wsb, None)  # noqa: E731
else:
    fn = lambda: L.jr_conv2d_bwd_filter(ctypes.byref(d), dt, x.data_ptr(), dy.data_ptr(), dw.data_ptr(), ws.data_ptr(), wsb, None)  # noqa: E731
_ffi.check("warm", fn())
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    fn()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / reps * 1e3
macs = n * ho * wo * co * kh * kw * ci
print(f"{layer} dt{dt} op{op}: {us:.1f} us  {2 * macs / us / 1e6:.1f} TF/s (fp32-equiv / bf16)", flush=True)
