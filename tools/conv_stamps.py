"""Per-block timeline of one conv GEMM launch from the stamps build
(`make -C jama16-retina-replication_amd/csrc stamps` -> jr/libjr_stamps.so;
Stamps in jr_conv_impl.h): where a block's cycles go (prologue = ring fill up
to the first barrier, K loop, of which vmcnt waits + barriers, epilogue), how
many blocks share a CU over the launch, and the clock the chip held.
Diagnostic only (the stamps cost a few % of the loop).
  python tools/conv_stamps.py <dtype 0|1|2|3> <op 0|1|2> <layer> <cfg> [reps]"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(HERE, "..", "jama16-retina-replication_amd")
os.environ.setdefault("JR_LIB_DIAG", os.path.join(PKG, "jr", "libjr_stamps.so"))
sys.path.insert(0, PKG)
sys.path.insert(0, HERE)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from jr import _ffi  # noqa: E402

LAYERS = {"c17x7": (64, 17, 17, 192, 192, 1, 7, 1, 0, 3), "c17x1": (64, 17, 17, 768, 192, 1, 1, 1, 0, 0),
          "c35x3": (64, 35, 35, 64, 96, 3, 3, 1, 1, 1), "c8x3": (64, 8, 8, 384, 384, 1, 3, 1, 0, 1),
          "conv5": (64, 73, 73, 80, 192, 3, 3, 1, 0, 0), "conv3": (64, 147, 147, 32, 64, 3, 3, 1, 1, 1),
          "c8x33": (64, 8, 8, 448, 384, 3, 3, 1, 1, 1), "m17": (64, 17, 17, 768, 512, 1, 1, 1, 0, 0),
          "c35x5": (64, 35, 35, 48, 64, 5, 5, 1, 2, 2), "c8x1": (64, 8, 8, 2048, 1152, 1, 1, 1, 0, 0)}


def main():
    dt, op, layer, cfg = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], int(sys.argv[4])
    reps = int(sys.argv[5]) if len(sys.argv) > 5 else 5
    _ffi.init(0)
    L = _ffi.load()
    L.jr_debug_set_stamps.restype = ctypes.c_int
    L.jr_debug_set_stamps.argtypes = [ctypes.c_void_p]
    n, h, w, ci, co, kh, kw, s, ph, pw = LAYERS[layer]
    ho, wo = (h + 2 * ph - kh) // s + 1, (w + 2 * pw - kw) // s + 1
    q = 8 if dt in (1, 3) else 4
    cs = (ci + q - 1) // q * q
    d = _ffi.ConvDesc(n, h, w, ci, co, kh, kw, s, s, ph, pw, ho, wo, 0, cs, 0, co)
    pl = 3 if dt == 3 else 1
    et = torch.bfloat16 if dt in (1, 3) else torch.float32
    x = torch.randn(pl * n * h * w * cs, device="cuda").to(et)
    wt = (torch.randn(pl * kh * kw * cs * co, device="cuda") * 0.05).to(et)
    dy = torch.randn(pl * n * ho * wo * co, device="cuda").to(et)
    ot = torch.bfloat16 if dt == 1 else torch.float32
    y = torch.zeros(n * ho * wo * co, device="cuda", dtype=ot)
    dx = torch.zeros(n * h * w * cs, device="cuda", dtype=ot)
    dw = torch.zeros(kh * kw * cs * co, device="cuda")
    wsb = 1 << 30
    ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
    for p in range(s * s if op == 1 else 1):
        _ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), op, dt, p, cfg))
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def run():
        if op == 0:
            return L.jr_conv2d_fwd(ctypes.byref(d), dt, P(x), P(wt), P(y), P(ws), wsb, None)
        if op == 1:
            return L.jr_conv2d_bwd_data(ctypes.byref(d), dt, P(dy), P(wt), P(dx), 0, P(ws), wsb, None)
        return L.jr_conv2d_bwd_filter(ctypes.byref(d), dt, P(x), P(dy), P(dw), P(ws), wsb, None)

    stamps = torch.zeros(8 * (1 << 21), dtype=torch.int64, device="cuda")
    for _ in range(reps):
        _ffi.check("warm", run())
    torch.cuda.synchronize()
    L.jr_debug_set_stamps(P(stamps))
    _ffi.check("stamped", run())
    torch.cuda.synchronize()
    L.jr_debug_set_stamps(None)
    st = stamps.view(-1, 8).cpu().numpy().astype(np.int64)
    st = st[st[:, 1] > 0]
    nb = len(st)
    r0, r1 = st[:, 0], st[:, 1]
    wall = (r1.max() - r0.min()) * 10e-3          # 100 MHz ticks -> us
    cyc = st[:, 2] + st[:, 3] + st[:, 4]
    dur = (r1 - r0) * 10e-3
    clock = np.median(cyc / np.maximum(r1 - r0, 1)) * 100e6 / 1e9
    hw, xcc = st[:, 6], st[:, 7] & 0xF
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 0x1
    se = (hw >> 13) & 0x7
    cu_key = xcc * 1000 + se * 100 + sh * 16 + cu
    ncu = len(np.unique(cu_key))
    busy = dur.sum() / (wall * ncu)
    print(f"{layer} dtype {dt} op {op} cfg {cfg}: {nb} blocks on {ncu} CUs, launch {wall:.1f} us, "
          f"clock {clock:.2f} GHz, mean resident blocks per CU {busy:.2f}")
    for name, v in (("block duration us", dur), ("prologue kcyc", st[:, 2] / 1e3), ("K loop kcyc", st[:, 3] / 1e3),
                    ("  waits+barriers kcyc", st[:, 5] / 1e3), ("epilogue kcyc", st[:, 4] / 1e3)):
        print(f"  {name:22s} mean {v.mean():8.2f}  p10 {np.percentile(v, 10):8.2f}  p50 {np.median(v):8.2f}  "
              f"p90 {np.percentile(v, 90):8.2f}  max {v.max():8.2f}")
    tot = cyc.sum()
    print(f"  share of block cycles: prologue {st[:, 2].sum() / tot:.3f}  loop {st[:, 3].sum() / tot:.3f} "
          f"(waits {st[:, 5].sum() / tot:.3f})  epilogue {st[:, 4].sum() / tot:.3f}")
    # start skew: how the blocks enter over the launch
    t = (r0 - r0.min()) * 10e-3
    print(f"  block start times us: p10 {np.percentile(t, 10):.1f} p50 {np.median(t):.1f} p90 {np.percentile(t, 90):.1f}"
          f"  last end {wall:.1f}")
    blocks_per_cu = np.bincount(np.unique(cu_key, return_inverse=True)[1])
    print(f"  blocks per CU: min {blocks_per_cu.min()} mean {blocks_per_cu.mean():.2f} max {blocks_per_cu.max()}")


if __name__ == "__main__":
    main()
