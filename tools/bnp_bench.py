"""Diagnostic: cost of the BN-backward partials in the data-gradient GEMM.

python tools/bnp_bench.py [f32x8|bf16]

Per Inception-v3 layer shape (B = 64, 299^2 geometry): µs of
jr_conv2d_bwd_data vs jr_conv2d_bwd_data_bnp (same tiles), and of the BN
backward it feeds, jr_bn_relu_bwd_multi (reduce + finalize + apply) vs
jr_bn_relu_bwd_parts (finalize + apply): whether the epilogue work costs
less than the reduce pass it removes.
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jama16-retina-replication_amd"))
import torch  # noqa: E402

from jr import _ffi  # noqa: E402

_ffi.init(0)
L = _ffi.load()
dtype = sys.argv[1] if len(sys.argv) > 1 else "bf16"
DT = {"f32x8": 2, "bf16": 1, "f32": 0}[dtype]
BDT = 1 if dtype == "bf16" else 0
TD = torch.bfloat16 if dtype == "bf16" else torch.float32
B = 64
# (h, c_in = dx channels, c_out, kh, kw, stride, pad) of consumer convs whose dgrad writes a BN layer's dy
SHAPES = [(147, 32, 64, 3, 3, 1, 1), (35, 64, 96, 3, 3, 1, 1), (35, 48, 64, 5, 5, 1, 2),
          (17, 160, 160, 1, 7, 1, 3), (17, 192, 192, 7, 1, 1, 3), (17, 768, 192, 1, 1, 1, 0),
          (8, 448, 384, 3, 3, 1, 1), (35, 288, 384, 3, 3, 2, 0)]
KEEP = []


def T(n, dt=TD):
    t = torch.randn(int(n), device="cuda").to(dt)
    KEEP.append(t)
    return t


def timeit(fn, n=30):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


tot = [0.0] * 4
for h, cin, cout, kh, kw, s, p in SHAPES:
    ho = (h + 2 * p - kh) // s + 1
    d = _ffi.ConvDesc(B, h, h, cin, cout, kh, kw, s, s, p, p, ho, ho, 0, cin, 0, cout)
    dy, w = T(B * ho * ho * cout), T(kh * kw * cin * cout)
    dx, raw = T(B * h * h * cin), T(B * h * h * cin)
    mean, inv, beta = T(cin, torch.float32), T(cin, torch.float32).abs() + 0.5, T(cin, torch.float32)
    P = ctypes.c_int32(0)
    if L.jr_conv2d_bwd_data_bnp_slots(ctypes.byref(d), DT, ctypes.byref(P)) != 0:
        print(f"{h}x{h} {cin}<-{cout}: unsupported")
        continue
    P = P.value
    part = torch.zeros(2 * cin * P, dtype=torch.float64, device="cuda")
    seg = (_ffi.BnpSeg * 1)(_ffi.BnpSeg(raw.data_ptr(), mean.data_ptr(), inv.data_ptr(), beta.data_ptr(),
                                        part.data_ptr(), 0, cin, 0, cin, cin, 0))
    wsb = L.jr_conv2d_workspace_size(ctypes.byref(d), 1, DT) + (1 << 20)
    m = B * h * h
    wsb = max(wsb, L.jr_bn_workspace_size(m, cin))
    ws = torch.zeros(wsb // 4 + 4, device="cuda")
    dbeta = torch.zeros(cin, device="cuda")
    out = T(m * cin)
    bseg = _ffi.BnSeg(dx.data_ptr(), 0, cin, cin, beta.data_ptr(), dbeta.data_ptr())
    a = timeit(lambda: L.jr_conv2d_bwd_data(ctypes.byref(d), DT, dy.data_ptr(), w.data_ptr(), dx.data_ptr(), 0,
                                            ws.data_ptr(), wsb, None))
    b = timeit(lambda: L.jr_conv2d_bwd_data_bnp(ctypes.byref(d), DT, dy.data_ptr(), w.data_ptr(), dx.data_ptr(), 0,
                                                1, ctypes.byref(seg), ws.data_ptr(), wsb, None))
    c = timeit(lambda: L.jr_bn_relu_bwd_multi(BDT, 1, ctypes.byref(bseg), raw.data_ptr(), 0, cin, m, cin,
                                              mean.data_ptr(), inv.data_ptr(), out.data_ptr(), ws.data_ptr(), wsb,
                                              None))
    e = timeit(lambda: L.jr_bn_relu_bwd_parts(BDT, 1, ctypes.byref(bseg), part.data_ptr(), P, raw.data_ptr(), 0, cin,
                                              m, cin, mean.data_ptr(), inv.data_ptr(), out.data_ptr(), ws.data_ptr(),
                                              wsb, None))
    cfg = L.jr_conv2d_get_config(ctypes.byref(d), 1, DT, 0)
    print(f"{h:3d}^2 {cin:4d}<-{cout:4d} {kh}x{kw}/{s} cfg {cfg:5d} P {P:6d}: dgrad {a:7.1f} -> {b:7.1f} us (+{b - a:5.1f})"
          f" | bn bwd {c:7.1f} -> {e:7.1f} us ({e - c:+6.1f}) | net {b - a + e - c:+6.1f}")
    for i, v in enumerate((a, b, c, e)):
        tot[i] += v
print(f"total: dgrad {tot[0]:.1f} -> {tot[1]:.1f}, bn bwd {tot[2]:.1f} -> {tot[3]:.1f}, "
      f"net {tot[1] - tot[0] + tot[3] - tot[2]:+.1f} us")
