"""Diagnostic: time the pooling kernels on the Inception-v3 pool shapes
(B=64, 299^2) for the libjr named by $JR_LIB; per-shape µs, algorithmic
GB/s and the per-step totals.   python tools/poolbench.py [f32|bf16]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jama16-retina-replication_amd"))
import torch  # noqa: E402

from jr import _ffi  # noqa: E402

_ffi.init(0)
L = _ffi.load()
DT = _ffi.JR_BF16 if len(sys.argv) > 1 and sys.argv[1] == "bf16" else _ffi.JR_F32
TD = torch.bfloat16 if DT == _ffi.JR_BF16 else torch.float32
B = 64
MAXP = [(147, 64), (71, 192), (35, 288), (17, 768)]
AVGP = [(35, 192), (35, 256), (35, 288), (17, 768), (17, 768), (17, 768), (17, 768), (8, 1280), (8, 2048)]


def timeit(fn, n=int(os.environ.get("POOLBENCH_N", "50"))):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
tot = {"maxpool fwd": 0.0, "maxpool bwd": 0.0, "avgpool fwd": 0.0, "avgpool bwd": 0.0}
for h, c in MAXP:
    ho = (h - 3) // 2 + 1
    d = _ffi.PoolDesc(B, h, h, c, ho, ho, 0, c, 0, c)
    x = torch.randn(B * h * h * c, device="cuda").relu().to(TD)
    y = torch.empty(B * ho * ho * c, device="cuda", dtype=TD)
    am = torch.empty(B * ho * ho * c, device="cuda", dtype=torch.uint8)
    dx = torch.empty_like(x)
    es = x.element_size()
    f = timeit(lambda: _ffi.check("mp", L.jr_maxpool3x3s2_fwd(ctypes.byref(d), DT, P(x), P(y), P(am), None)))
    b = timeit(lambda: _ffi.check("mpb", L.jr_maxpool3x3s2_bwd(ctypes.byref(d), DT, P(am), P(y), P(dx), 0, None)))
    nf = (x.numel() + y.numel()) * es + am.numel()
    tot["maxpool fwd"] += f
    tot["maxpool bwd"] += b
    print(f"maxpool {h:3d}^2 x {c:4d}: fwd {f:7.1f} us {nf / f / 1e3:6.0f} GB/s | bwd {b:7.1f} us {nf / b / 1e3:6.0f} GB/s")
for h, c in AVGP:
    d = _ffi.PoolDesc(B, h, h, c, h, h, 0, c, 0, c)
    x = torch.randn(B * h * h * c, device="cuda").to(TD)
    y = torch.empty_like(x)
    n = 2 * x.numel() * x.element_size()
    f = timeit(lambda: _ffi.check("ap", L.jr_avgpool3x3s1_fwd(ctypes.byref(d), DT, P(x), P(y), None)))
    b = timeit(lambda: _ffi.check("apb", L.jr_avgpool3x3s1_bwd(ctypes.byref(d), DT, P(x), P(y), 0, None)))
    tot["avgpool fwd"] += f
    tot["avgpool bwd"] += b
    print(f"avgpool {h:3d}^2 x {c:4d}: fwd {f:7.1f} us {n / f / 1e3:6.0f} GB/s | bwd {b:7.1f} us {n / b / 1e3:6.0f} GB/s")
print("per step: " + ", ".join(f"{k} {v:.1f} us" for k, v in tot.items()) +
      f"  [{os.path.basename(_ffi.LIB_PATH)}]")
