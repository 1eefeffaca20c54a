"""Where does a small conv GEMM's time go: fixed per-launch cost or per-K-tile
cost?  Times a 1x1 conv at 17^2, B=64 (M = 18,496; N = c_out) for growing
c_in (= K) with a fixed tile and no split-K, so time(K) = intercept (launch,
ring fill, epilogue) + slope x K-tiles.  Also times the same GEMM at 8^2 and
35^2 and an empty-ish K (c_in = 8 / 16).

  python tools/ksweep_probe.py [dtype 1 = bf16 | 2 = x8] [cfg,cfg,...]
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jama16-retina-replication_amd"))
import torch  # noqa: E402
from jr import _ffi  # noqa: E402

DT = int(sys.argv[1]) if len(sys.argv) > 1 else 1
CFGS = [int(c) for c in sys.argv[2].split(",")] if len(sys.argv) > 2 else ([3, 0, 5] if DT == 1 else [3, 0, 11])
_ffi.init(0)
L = _ffi.load()
et = torch.bfloat16 if DT == 1 else torch.float32
B = 64


def t_gemm(h, cin, cout, cfg, reps=30):
    d = _ffi.ConvDesc(B, h, h, cin, cout, 1, 1, 1, 1, 0, 0, h, h, 0, cin, 0, cout)
    x = torch.randn(B * h * h * cin, device="cuda").to(et)
    w = (torch.randn(cin * cout, device="cuda") * 0.05).to(et)
    y = torch.zeros(B * h * h * cout, device="cuda", dtype=et)
    wsb = L.jr_conv2d_workspace_size(ctypes.byref(d), 0, DT)
    ws = torch.zeros(wsb // 4 + 64, device="cuda")
    _ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), 0, DT, 0, cfg | (1 << 8)))
    try:
        f = lambda: L.jr_conv2d_fwd(ctypes.byref(d), DT, x.data_ptr(), w.data_ptr(), y.data_ptr(),  # noqa: E731
                                    ws.data_ptr(), wsb, None)
        for _ in range(3):
            _ffi.check("fwd", f())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3
    finally:
        L.jr_conv2d_set_config(ctypes.byref(d), 0, DT, 0, -1)


print(f"dtype {DT}, 1x1 conv fwd, B={B}, no split-K; us per launch (back-to-back, one stream)")
for h, cout in ((17, 192), (8, 384), (35, 96)):
    for cfg in CFGS:
        row = []
        for cin in (16, 64, 128, 256, 512, 768, 1024, 1536, 2048):
            row.append(f"{cin}:{t_gemm(h, cin, cout, cfg):6.1f}")
        print(f"{h}^2 c_out {cout} cfg {cfg:2d}  " + "  ".join(row), flush=True)
