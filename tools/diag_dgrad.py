"""Diagnostic: repeat one bf16 conv dgrad (conv2d_5 geometry, B=2) and locate
any element that differs from the fp64 oracle or between repeats.

  python tools/diag_dgrad.py [reps]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jama16-retina-replication_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import tf_ops as R  # noqa: E402
import test_gpu_bf16 as T  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    ffi = T._lib()
    L = ffi.load()
    n, h, w, cin, cout, kh, kw, s, pad = (2, 73, 73, 80, 192, 3, 3, 1, "valid")
    rng = np.random.default_rng(1)
    x = T.bf16_round(rng.standard_normal((n, h, w, cin)))
    wt32 = (rng.standard_normal((kh, kw, cin, cout)) / np.sqrt(kh * kw * cin)).astype(np.float32)
    wt = T.bf16_round(wt32)
    d, ho, wo = T._desc(ffi, n, h, w, cin, cout, kh, kw, s, pad, cin)
    hwio, _ = T._weights(ffi, L, wt32)
    dy = T.bf16_round(rng.standard_normal((n, ho, wo, cout)))
    DY = T.dev_bf16(dy)
    torch.cuda.synchronize()
    ref = R.conv2d_bwd_data(dy, wt, x.shape, s, pad)
    wsb = L.jr_conv2d_workspace_size(ctypes.byref(d), 1, 1)
    ws = torch.full((wsb // 4 + 4,), float("nan"), device="cuda")
    print("cfg", L.jr_conv2d_get_config(ctypes.byref(d), 1, 1, 0), "ws", wsb, flush=True)
    first = None
    for r in range(reps):
        DX = torch.full((x.size,), 3.0, dtype=torch.bfloat16, device="cuda")
        torch.cuda.synchronize()
        ffi.check("dgrad", L.jr_conv2d_bwd_data(ctypes.byref(d), 1, DY.data_ptr(), hwio.data_ptr(), DX.data_ptr(),
                                                0, ws.data_ptr(), wsb, None))
        got = T.host(DX).reshape(x.shape)
        err = np.abs(got - ref) / np.max(np.abs(ref))
        bad = np.argwhere(err > 8e-3)
        same = first is None or np.array_equal(got, first)
        if first is None:
            first = got
        print(f"rep {r}: relerr {err.max():.3e} bad {len(bad)} equal_to_first {same}", flush=True)
        if len(bad):
            b, hh, ww, c = bad[:, 0], bad[:, 1], bad[:, 2], bad[:, 3]
            print("   b", np.unique(b), "h", np.unique(hh)[:20], "w", np.unique(ww)[:20], "c", np.unique(c)[:40])
            print("   sample got/ref", [(float(got[tuple(i)]), float(ref[tuple(i)])) for i in bad[:5]])


if __name__ == "__main__":
    main()
