"""Probe: fp32 convolutions on the matrix cores with a
fp16 three-way split and SIX f16 MFMAs per product (jr_debug_x8_f16) against
the shipping JR_F32_X8 (bf16 split, eight MFMAs), same tile, one GEMM at a
time: time per call (interleaved) and error vs an fp64 reference, with the
fp32-MFMA kernel (JR_F32) as the fp32 yardstick.  Gate: error within x8's
class and >= 15 % faster per GEMM.
Historical: ran at eb5182a (profiles/r06_x6h_probe.txt); its debug entry point
jr_debug_x8_f16 was removed once the split shipped as JR_F32_X6H (dtype 4,
tests/test_gpu_x6h.py), so it no longer runs against the current libjr.
  python tools/probes/x6h_probe.py [reps]"""
import ctypes
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "jama16-retina-replication_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from jr import _ffi  # noqa: E402

LAYERS = {"conv5": (64, 73, 73, 80, 192, 3, 3, 1, 0, 0), "conv3": (64, 147, 147, 32, 64, 3, 3, 1, 1, 1),
          "m17": (64, 17, 17, 768, 512, 1, 1, 1, 0, 0), "m8": (64, 8, 8, 448, 384, 3, 3, 1, 1, 1),
          "c17x7": (64, 17, 17, 192, 192, 1, 7, 1, 0, 3), "c35x3": (64, 35, 35, 64, 96, 3, 3, 1, 1, 1),
          "mixed3": (64, 35, 35, 288, 384, 3, 3, 2, 0, 0)}
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
_ffi.init(0)
L = _ffi.load()
X8, F32 = 2, 0


def pow2_scale(t):
    m = float(t.abs().max())
    return 1.0 if m == 0 else 2.0 ** (14 - math.floor(math.log2(m)))


for name, (n, h, w, ci, co, kh, kw, s, ph, pw) in LAYERS.items():
    ho, wo = (h + 2 * ph - kh) // s + 1, (w + 2 * pw - kw) // s + 1
    d = _ffi.ConvDesc(n, h, w, ci, co, kh, kw, s, s, ph, pw, ho, wo, 0, ci, 0, co)
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.relu(torch.randn(n, h, w, ci, device="cuda", generator=g))                  # BN+ReLU-like
    wt = torch.randn(kh, kw, ci, co, device="cuda", generator=g) * math.sqrt(2.0 / (kh * kw * ci))
    dy = torch.randn(n, ho, wo, co, device="cuda", generator=g) * 1e-5                   # a gradient
    xd, wd, dyd = x.double().permute(0, 3, 1, 2), wt.double().permute(3, 2, 0, 1), dy.double().permute(0, 3, 1, 2)
    refs = [F.conv2d(xd, wd, stride=s, padding=(ph, pw)).permute(0, 2, 3, 1),
            torch.nn.grad.conv2d_input(xd.shape, wd, dyd, stride=s, padding=(ph, pw)).permute(0, 2, 3, 1),
            torch.nn.grad.conv2d_weight(xd, wd.shape, dyd, stride=s, padding=(ph, pw)).permute(2, 3, 1, 0)]
    wsb = max(L.jr_conv2d_workspace_size(ctypes.byref(d), o, dt) for o in range(3) for dt in (X8, F32)) * 2
    ws = torch.zeros(wsb // 4 + 4, device="cuda")
    for op in range(3):
        if op == 1 and s > 1:
            continue        # (stride-2 data gradient: four phase GEMMs; fwd / wgrad suffice here)
        cfg = L.jr_conv2d_get_config(ctypes.byref(d), op, X8, 0)
        tile = cfg & 255
        if 28 <= tile < 42:
            cfg = (cfg & ~255) | (tile - 28)          # the same tile without stream-K
        elif 14 <= tile < 28:
            cfg = (cfg & ~255) | (tile - 14)          # the x8 kernel of that tile
        for ph_ in range(s * s if op == 1 else 1):
            _ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), op, X8, ph_, cfg))
        sa, sb = [(pow2_scale(x), pow2_scale(wt)), (pow2_scale(dy), pow2_scale(wt)), (pow2_scale(x), pow2_scale(dy))][op]
        out = torch.zeros(refs[op].shape, dtype=torch.float32, device="cuda")

        def run(dt):
            if op == 0:
                return L.jr_conv2d_fwd(ctypes.byref(d), dt, x.data_ptr(), wt.data_ptr(), out.data_ptr(), ws.data_ptr(),
                                       wsb, None)
            if op == 1:
                return L.jr_conv2d_bwd_data(ctypes.byref(d), dt, dy.data_ptr(), wt.data_ptr(), out.data_ptr(), 0,
                                            ws.data_ptr(), wsb, None)
            return L.jr_conv2d_bwd_filter(ctypes.byref(d), dt, x.data_ptr(), dy.data_ptr(), out.data_ptr(),
                                          ws.data_ptr(), wsb, None)
        res = {}
        for variant, dt, on in (("f32", F32, 0), ("x8", X8, 0), ("h6", X8, 1)):
            L.jr_debug_x8_f16(on, sa, sb)
            _ffi.check(variant, run(dt))
            torch.cuda.synchronize()
            ref = refs[op]
            res[variant] = {"err": float((out.double() - ref).abs().max() / ref.abs().max())}
        times = {"x8": [], "h6": []}
        for _ in range(3):
            for variant, on in (("x8", 0), ("h6", 1)):
                L.jr_debug_x8_f16(on, sa, sb)
                run(X8)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    run(X8)
                e1.record()
                torch.cuda.synchronize()
                times[variant].append(e0.elapsed_time(e1) / reps * 1e3)
        L.jr_debug_x8_f16(0, 1.0, 1.0)
        for ph_ in range(s * s if op == 1 else 1):
            _ffi.check("reset", L.jr_conv2d_set_config(ctypes.byref(d), op, X8, ph_, -1))
        t8, t6 = min(times["x8"]), min(times["h6"])
        print(f"{name:7s} {['fwd', 'dgrad', 'wgrad'][op]:5s} cfg {cfg:5d}  x8 {t8:8.1f} us  h6 {t6:8.1f} us  "
              f"({(t8 / t6 - 1) * 100:+5.1f} % faster)  err vs fp64: f32 {res['f32']['err']:.2e}  x8 "
              f"{res['x8']['err']:.2e}  h6 {res['h6']['err']:.2e}", flush=True)
