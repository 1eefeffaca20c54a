"""Time one conv op of an Inception layer under EVERY tile config and several
split-K factors (jr_conv2d_set_config), HIP events over `reps` back-to-back
calls, FWD with the fused BN statistics as the engine runs it.  Shows what
jr_conv2d_autotune's two-pass search (every tile at the planner's split, then
other splits for the three fastest tiles) may miss.
  python tools/conv_sweep.py <dtype 0|1|2|3> <op 0|1|2> <layer> [reps]
layers: c17x7 (17^2 192->192 1x7 same), c17x1 (17^2 768->192 1x1), c35x3 (35^2 64->96 3x3 same),
        c8x3 (8^2 384->384 1x3 same), conv5 (73^2 80->192 3x3 valid), conv1 (299^2 3->32 3x3/2 valid),
        conv2 (149^2 32->32 3x3 valid), conv3 (147^2 32->64 3x3 same)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jama16-retina-replication_amd"))
import torch  # noqa: E402
from jr import _ffi  # noqa: E402

# n, h, w, cin, cout, kh, kw, stride, ph, pw
LAYERS = {"c17x7": (64, 17, 17, 192, 192, 1, 7, 1, 0, 3), "c17x1": (64, 17, 17, 768, 192, 1, 1, 1, 0, 0),
          "c35x3": (64, 35, 35, 64, 96, 3, 3, 1, 1, 1), "c8x3": (64, 8, 8, 384, 384, 1, 3, 1, 0, 1),
          "conv5": (64, 73, 73, 80, 192, 3, 3, 1, 0, 0), "conv1": (64, 299, 299, 3, 32, 3, 3, 2, 0, 0),
          "conv2": (64, 149, 149, 32, 32, 3, 3, 1, 0, 0), "conv3": (64, 147, 147, 32, 64, 3, 3, 1, 1, 1),
          "c17x7v": (64, 17, 17, 192, 192, 7, 1, 1, 3, 0), "c8x3v": (64, 8, 8, 384, 384, 3, 1, 1, 1, 0),
          "c8x33": (64, 8, 8, 448, 384, 3, 3, 1, 1, 1), "c35x33": (64, 35, 35, 96, 96, 3, 3, 1, 1, 1),
          "c35p192": (64, 35, 35, 192, 32, 1, 1, 1, 0, 0), "c35p288": (64, 35, 35, 288, 64, 1, 1, 1, 0, 0)}
dt, op, layer = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
_ffi.init(0)
L = _ffi.load()
n, h, w, ci, co, kh, kw, s, ph, pw = LAYERS[layer]
ho, wo = (h + 2 * ph - kh) // s + 1, (w + 2 * pw - kw) // s + 1
q = 8 if dt in (1, 3) else 4
cs = (ci + q - 1) // q * q
d = _ffi.ConvDesc(n, h, w, ci, co, kh, kw, s, s, ph, pw, ho, wo, 0, cs, 0, co)
pl = 3 if dt == 3 else 1
et = torch.bfloat16 if dt in (1, 3) else torch.float32
ot = torch.bfloat16 if dt == 1 else torch.float32
x = torch.randn(pl * n * h * w * cs, device="cuda").to(et)
wt = (torch.randn(pl * kh * kw * cs * co, device="cuda") * 0.05).to(et)
dy = torch.randn(pl * n * ho * wo * co, device="cuda").to(et)
y = torch.zeros(n * ho * wo * co, device="cuda", dtype=ot)
dx = torch.zeros(n * h * w * cs, device="cuda", dtype=ot)
dw = torch.zeros(kh * kw * cs * co, device="cuda")
mean, inv = torch.zeros(co, device="cuda"), torch.zeros(co, device="cuda")
wsb = 1 << 30
ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731


def run():
    if op == 0:
        return L.jr_conv2d_fwd_bn_stats(ctypes.byref(d), dt, P(x), P(wt), P(y), ctypes.c_float(1e-3), P(mean), P(inv),
                                        P(ws), wsb, None)
    if op == 1:
        return L.jr_conv2d_bwd_data(ctypes.byref(d), dt, P(dy), P(wt), P(dx), 0, P(ws), wsb, None)
    return L.jr_conv2d_bwd_filter(ctypes.byref(d), dt, P(x), P(dy), P(dw), P(ws), wsb, None)


flops = 2.0 * n * ho * wo * co * kh * kw * ci
nph = s * s if op == 1 else 1
res = []
for tile in range(L.jr_conv2d_num_configs(dt)):
    for sp in (1, 2, 3, 4, 6, 8, 12, 16, 32, 64, 128, 256, 512, 1024):
        cfg = tile | (sp << 8)
        ok = all(L.jr_conv2d_set_config(ctypes.byref(d), op, dt, p, cfg) == 0 for p in range(nph))
        if not ok or (L.jr_conv2d_get_config(ctypes.byref(d), op, dt, 0) & 255) != tile or run() != 0:
            continue        # (a halo config this geometry does not take falls back: skipped)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / reps * 1e3
        res.append((t, tile, sp))
for p in range(nph):
    L.jr_conv2d_set_config(ctypes.byref(d), op, dt, p, -1)
auto = L.jr_conv2d_get_config(ctypes.byref(d), op, dt, 0)
res.sort()
print(f"{layer} dtype {dt} op {op}: heuristic cfg tile {auto & 255} splits {auto >> 8}")
for t, tile, sp in res[:12]:
    print(f"  tile {tile:2d} splits {sp:3d}: {t:8.1f} us  {flops / t / 1e6:7.1f} TF/s")
