"""VERDICT r04 item 3 probe: would storing bf16 conv inputs at a 64-aligned
channel stride (zero pad channels, zero filter rows) make the GEMMs faster?

For each Inception-v3 layer whose input channel count is not a multiple of
64 (conv5's 80, the 35^2 branches' 48 / 96 / 288, the 17^2 branches' 160),
at B=64, times the layer's three GEMMs (fwd, dgrad, wgrad) with the real
c_in and with c_in padded to the next multiple of 64 (and to 32 where that
differs), each autotuned over every tile / split / stream-K config of the
dtype (jr_conv2d_autotune), then 20 timed launches of the winner.

  python tools/pad_probe.py [dtype: 1 = bf16 (default), 2 = x8]
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jama16-retina-replication_amd"))
import torch  # noqa: E402
from jr import _ffi  # noqa: E402

DT = int(sys.argv[1]) if len(sys.argv) > 1 else 1
LAYERS = [  # name, h, w, cin, cout, kh, kw, stride, pad_h, pad_w
    ("conv5 3x3 73^2", 73, 73, 80, 192, 3, 3, 1, 0, 0),
    ("35^2 5x5 48->64", 35, 35, 48, 64, 5, 5, 1, 2, 2),
    ("35^2 3x3 96->96", 35, 35, 96, 96, 3, 3, 1, 1, 1),
    ("35^2 1x1 288->64", 35, 35, 288, 64, 1, 1, 1, 0, 0),
    ("mixed3 3x3/2 288->384", 35, 35, 288, 384, 3, 3, 2, 0, 0),
    ("17^2 1x7 160->160", 17, 17, 160, 160, 1, 7, 1, 0, 3),
    ("17^2 7x1 160->192", 17, 17, 160, 192, 7, 1, 1, 3, 0),
]
B = 64
_ffi.init(0)
L = _ffi.load()
et = torch.bfloat16 if DT == 1 else torch.float32
ot = torch.bfloat16 if DT == 1 else torch.float32


def run(d, op, x, w, y, ws, wsb, cfg=None):
    if op == 0:
        return L.jr_conv2d_fwd(ctypes.byref(d), DT, x.data_ptr(), w.data_ptr(), y.data_ptr(), ws.data_ptr(), wsb, None)
    if op == 1:
        return L.jr_conv2d_bwd_data(ctypes.byref(d), DT, x.data_ptr(), w.data_ptr(), y.data_ptr(), 0, ws.data_ptr(),
                                    wsb, None)
    return L.jr_conv2d_bwd_filter(ctypes.byref(d), DT, x.data_ptr(), w.data_ptr(), y.data_ptr(), ws.data_ptr(), wsb,
                                  None)


def time_layer(h, w, cin, cout, kh, kw, s, ph, pw):
    ho, wo = (h + 2 * ph - kh) // s + 1, (w + 2 * pw - kw) // s + 1
    d = _ffi.ConvDesc(B, h, w, cin, cout, kh, kw, s, s, ph, pw, ho, wo, 0, cin, 0, cout)
    x = torch.randn(B * h * w * cin, device="cuda").to(et)
    wt = (torch.randn(kh * kw * cin * cout, device="cuda") * 0.05).to(et)
    dy = torch.randn(B * ho * wo * cout, device="cuda").to(et)
    y = torch.zeros(B * ho * wo * cout, device="cuda", dtype=ot)
    dx = torch.zeros(B * h * w * cin, device="cuda", dtype=ot)
    dw = torch.zeros(kh * kw * cin * cout, device="cuda")
    wsb = max(L.jr_conv2d_workspace_size(ctypes.byref(d), op, DT) for op in range(3))
    ws = torch.zeros(wsb // 4 + 64, device="cuda")
    out = []
    for op, (a, b, c) in enumerate(((x, wt, y), (dy, wt, dx), (x, dy, dw))):
        _ffi.check("autotune", L.jr_conv2d_autotune(ctypes.byref(d), op, DT, a.data_ptr(), b.data_ptr(), c.data_ptr(),
                                                    ws.data_ptr(), wsb, None))
        for _ in range(3):
            _ffi.check("run", run(d, op, a, b, c, ws, wsb))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run(d, op, a, b, c, ws, wsb)
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) / 20 * 1e3)
        cfgs = [L.jr_conv2d_get_config(ctypes.byref(d), op, DT, 0)]
        out.append(cfgs[0])
    return out


print(f"dtype {DT}, B={B}: per GEMM us (config id) for the real c_in and padded strides")
for name, h, w, cin, cout, kh, kw, s, ph, pw in LAYERS:
    pads = sorted({cin, (cin + 31) // 32 * 32, (cin + 63) // 64 * 64})
    for cp in pads:
        r = time_layer(h, w, cp, cout, kh, kw, s, ph, pw)
        macs = B * ((h + 2 * ph - kh) // s + 1) * ((w + 2 * pw - kw) // s + 1) * cout * kh * kw * cin
        tot = r[0] + r[2] + r[4]
        print(f"{name:24s} c_in {cin:4d} stored {cp:4d}: fwd {r[0]:7.1f} ({r[1]:5d})  dgrad {r[2]:7.1f} ({r[3]:5d})  "
              f"wgrad {r[4]:7.1f} ({r[5]:5d})  sum {tot:7.1f} us  {6 * macs / tot / 1e6:6.1f} TF/s (real MACs)",
              flush=True)
