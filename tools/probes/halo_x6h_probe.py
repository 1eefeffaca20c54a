"""Probe: the JR_F32_X6H halo-tiled forward (kHaloF32 ids 42..50) against the
x6h implicit GEMM's pinned pick, per layer geometry of the bench workload
(B = 64), interleaved timing, same scales.
  python tools/probes/halo_x6h_probe.py [reps]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "jama16-retina-replication_amd"))
import torch  # noqa: E402
from jr import _ffi  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
_ffi.init(0)
L = _ffi.load()
X6H = 4
BASE = L.jr_conv2d_num_configs(2)
# (name, n, h, w, cin, cout, kh, kw, pad_h, pad_w, halo ids to try)
LAYERS = [("17x17 1x7 128->128", 64, 17, 17, 128, 128, 1, 7, 0, 3, [0, 6]),
          ("17x17 7x1 160->160", 64, 17, 17, 160, 160, 7, 1, 3, 0, [1, 7]),
          ("17x17 1x7 192->192", 64, 17, 17, 192, 192, 1, 7, 0, 3, [0, 6]),
          ("35x35 3x3 64->96", 64, 35, 35, 64, 96, 3, 3, 1, 1, [2, 3]),
          ("8x8 3x3 448->384", 64, 8, 8, 448, 384, 3, 3, 1, 1, [3]),
          ("8x8 1x3 384->384", 64, 8, 8, 384, 384, 1, 3, 0, 1, [4]),
          ("147x147 3x3 32->64", 64, 147, 147, 32, 64, 3, 3, 1, 1, [8])]
for name, n, h, w, ci, co, kh, kw, ph, pw, ids in LAYERS:
    d = _ffi.ConvDesc(n, h, w, ci, co, kh, kw, 1, 1, ph, pw, h, w, 0, ci, 0, co)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.relu(torch.randn(n * h * w * ci, device="cuda", generator=g))
    wt = torch.randn(kh * kw * ci * co, device="cuda", generator=g) * 0.05
    y = torch.zeros(n * h * w * co, device="cuda")
    st = torch.zeros(2 * co, device="cuda")
    d.x_bound, d.w_bound = 8.0, 0.5
    wsb = L.jr_conv2d_workspace_size(ctypes.byref(d), 0, X6H) * 2 + (64 << 20)
    ws = torch.zeros(wsb // 4, device="cuda")
    gemm = L.jr_conv2d_get_config(ctypes.byref(d), 0, X6H, 0)
    cands = [("gemm", -1)] + [(f"halo{i}", BASE + i) for i in ids]

    def run():
        _ffi.check("fwd", L.jr_conv2d_fwd_bn_stats(ctypes.byref(d), X6H, x.data_ptr(), wt.data_ptr(), y.data_ptr(),
                                                   1e-3, st.data_ptr(), st.data_ptr() + 4 * co, ws.data_ptr(), wsb,
                                                   None))
    best = {}
    for _ in range(3):
        for lab, cfg in cands:
            _ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), 0, X6H, 0, cfg))
            run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / reps * 1e3
            best[lab] = min(best.get(lab, 1e9), t)
    _ffi.check("reset", L.jr_conv2d_set_config(ctypes.byref(d), 0, X6H, 0, -1))
    print(f"{name:22s} gemm (heuristic cfg {gemm}) {best['gemm']:7.1f} us  " +
          "  ".join(f"{k} {v:7.1f} us" for k, v in best.items() if k != "gemm"), flush=True)
