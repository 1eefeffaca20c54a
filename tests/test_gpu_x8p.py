"""JR_F32_X8P parity: fp32 convolutions whose operands arrive pre-split into
three bf16 planes (jr_split_x8p, jr_conv_weights_x8p).

* The split is exact: h + m + l == x bit for bit (checked in fp64), with
  h = bf16_rn(x) and m = bf16_rn(x - h) — the terms of the in-register split
  of JR_F32_X8 (jr_conv.hip SplitFrag).
* The convolutions are held to the SAME fp32 tolerances as JR_F32 /
  JR_F32_X8 against the fp64 oracle (test_gpu_ops.py): 5e-6 of max|ref| for
  fwd / dgrad, 1e-5 for wgrad.
* With the same tile geometry and split-K factor (x8 tile 0 and x8p tile 0:
  128x128, BK 16, one split) X8P forms the same products in the same
  per-accumulator order as X8, so fwd, dgrad and wgrad are bitwise equal.
"""
import ctypes

import numpy as np
import pytest

from oracle import tf_ops as R

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

X8, X8P = 2, 3
_KEEP = []


@pytest.fixture(autouse=True)
def _keep_alive():
    yield
    torch.cuda.synchronize()
    _KEEP.clear()


def _lib():
    from jr import _ffi
    _ffi.init(0)
    return _ffi


def dev(a, dtype=torch.float32):
    t = torch.as_tensor(np.ascontiguousarray(a)).to("cuda", dtype=dtype)
    _KEEP.append(t)
    return t


def zeros(n, dtype=torch.float32):
    t = torch.zeros(int(n), dtype=dtype, device="cuda")
    _KEEP.append(t)
    return t


def host(t):
    torch.cuda.synchronize()
    return t.to(torch.float64).cpu().numpy() if t.dtype == torch.bfloat16 else t.cpu().numpy()


def relerr(got, ref):
    ref = np.asarray(ref, np.float64)
    return float(np.max(np.abs(got - ref)) / max(np.max(np.abs(ref)), 1e-30))


def split_planes(ffi, L, a, c_pad=None):
    """fp32 [rows][c] -> device bf16 planes [3][rows][c_pad] via jr_split_x8p."""
    a = np.ascontiguousarray(a, np.float32)
    c = a.shape[-1]
    rows = a.size // c
    c_pad = c_pad or c
    src = dev(a)
    ps = rows * c_pad
    dst = zeros(3 * ps, torch.bfloat16)
    ffi.check("split", L.jr_split_x8p(src.data_ptr(), rows, c, 0, c, dst.data_ptr(), c_pad, 0, c_pad, ps, None))
    return dst


def weight_planes(ffi, L, wt):
    kh, kw, cin, cout = wt.shape
    c8 = (cin + 7) // 8 * 8
    W = dev(wt)
    hw = zeros(3 * wt.size, torch.bfloat16)
    tt = zeros(3 * cout * kh * kw * c8, torch.bfloat16)
    ffi.check("wprep x8p", L.jr_conv_weights_x8p(W.data_ptr(), kh, kw, cin, cout, hw.data_ptr(), tt.data_ptr(), None))
    return W, hw, tt


def _desc(ffi, n, h, w, cin, cout, kh, kw, s, pad, x_stride=None):
    ph, pw = ((kh - 1) // 2, (kw - 1) // 2) if pad == "same" else (0, 0)
    ho, wo = (h + 2 * ph - kh) // s + 1, (w + 2 * pw - kw) // s + 1
    return ffi.ConvDesc(n, h, w, cin, cout, kh, kw, s, s, ph, pw, ho, wo, 0, x_stride or cin, 0, cout), ho, wo


def test_split_exact():
    ffi = _lib()
    L = ffi.load()
    rng = np.random.default_rng(5)
    a = (rng.standard_normal((777, 36)) * np.exp(rng.uniform(-20, 20, (777, 36)))).astype(np.float32)
    a[0, :4] = [0.0, -0.0, 1.0, np.float32(1 + 2 ** -23)]
    P = host(split_planes(ffi, L, a, c_pad=40)).reshape(3, 777, 40)
    h, m, l = P
    assert np.array_equal(h[:, :36] + m[:, :36] + l[:, :36], a.astype(np.float64))
    hb = torch.as_tensor(a).to(torch.bfloat16).to(torch.float64).numpy()
    assert np.array_equal(h[:, :36], hb)
    assert not P[:, :, 36:].any()
    # generic (non-vector) path: c = 3 padded to 8 (the conv1 image)
    img = rng.uniform(0, 1, (50, 3)).astype(np.float32)
    Q = host(split_planes(ffi, L, img, c_pad=8)).reshape(3, 50, 8)
    assert np.array_equal(Q[:, :, :3].sum(0), img.astype(np.float64)) and not Q[:, :, 3:].any()


def test_weight_planes_exact():
    ffi = _lib()
    L = ffi.load()
    rng = np.random.default_rng(6)
    for shape in [(3, 3, 3, 32), (1, 7, 160, 192), (5, 5, 48, 64)]:
        wt = rng.standard_normal(shape).astype(np.float32)
        kh, kw, cin, cout = shape
        c8 = (cin + 7) // 8 * 8
        _, hw, tt = weight_planes(ffi, L, wt)
        hwp = host(hw).reshape(3, *shape)
        assert np.array_equal(hwp.sum(0), wt.astype(np.float64))
        tp = host(tt).reshape(3, cout, kh, kw, c8)
        exp = np.zeros((cout, kh, kw, c8))
        exp[..., :cin] = wt.transpose(3, 0, 1, 2)
        assert np.array_equal(tp.sum(0), exp)


CASES = [
    (2, 35, 35, 192, 64, 1, 1, 1, "same"),
    (2, 35, 35, 48, 64, 5, 5, 1, "same"),
    (2, 17, 17, 128, 192, 1, 7, 1, "same"),
    (2, 17, 17, 160, 160, 7, 1, 1, "same"),
    (2, 35, 35, 288, 384, 3, 3, 2, "valid"),
    (3, 17, 17, 192, 320, 3, 3, 2, "valid"),
    (2, 8, 8, 448, 384, 3, 3, 1, "same"),
    (2, 8, 8, 384, 384, 1, 3, 1, "same"),
    (2, 73, 73, 80, 192, 3, 3, 1, "valid"),
    (2, 37, 37, 3, 32, 3, 3, 2, "valid"),     # conv1: image planes 8 channels wide
    (1, 29, 31, 32, 48, 3, 3, 1, "same"),     # ragged M / N tails
]


def _run(ffi, L, case, seed, cfg=None, extra_ws=0):
    n, h, w, cin, cout, kh, kw, s, pad = case
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((n, h, w, cin)).astype(np.float32)
    wt = (rng.standard_normal((kh, kw, cin, cout)) / np.sqrt(kh * kw * cin)).astype(np.float32)
    c8 = (cin + 7) // 8 * 8
    d, ho, wo = _desc(ffi, n, h, w, cin, cout, kh, kw, s, pad, x_stride=c8)
    XP = split_planes(ffi, L, x.reshape(-1, cin), c_pad=c8)
    _, HW, WT = weight_planes(ffi, L, wt)
    wsb = max(L.jr_conv2d_workspace_size(ctypes.byref(d), op, X8P) for op in range(3)) + extra_ws
    ws = zeros(wsb // 4 + 4)
    if cfg is not None:
        for op in (0, 2):
            ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), op, X8P, 0, cfg))
        if cin % 8 == 0:
            for ph in range(s * s):
                ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), 1, X8P, ph, cfg))
    out = {}
    ref = R.conv2d(x, wt, s, pad)
    Y = zeros(ref.size)
    ffi.check("fwd", L.jr_conv2d_fwd(ctypes.byref(d), X8P, XP.data_ptr(), WT.data_ptr(), Y.data_ptr(),
                                     ws.data_ptr(), wsb, None))
    out["fwd"] = relerr(host(Y).reshape(ref.shape), ref)
    dy = rng.standard_normal(ref.shape).astype(np.float32)
    DYP = split_planes(ffi, L, dy.reshape(-1, cout))
    if cin % 8 == 0:
        ref_dx = R.conv2d_bwd_data(dy, wt, x.shape, s, pad)
        DX = zeros(x.size)
        ffi.check("dgrad", L.jr_conv2d_bwd_data(ctypes.byref(d), X8P, DYP.data_ptr(), HW.data_ptr(), DX.data_ptr(),
                                                0, ws.data_ptr(), wsb, None))
        out["dgrad"] = relerr(host(DX).reshape(x.shape), ref_dx)
        ffi.check("dgrad acc", L.jr_conv2d_bwd_data(ctypes.byref(d), X8P, DYP.data_ptr(), HW.data_ptr(),
                                                    DX.data_ptr(), 1, ws.data_ptr(), wsb, None))
        out["dgrad_acc"] = relerr(host(DX).reshape(x.shape), 2 * ref_dx)
    ref_dw = R.conv2d_bwd_filter(x, dy, wt.shape, s, pad)
    DW = zeros(wt.size)
    ffi.check("wgrad", L.jr_conv2d_bwd_filter(ctypes.byref(d), X8P, XP.data_ptr(), DYP.data_ptr(), DW.data_ptr(),
                                              ws.data_ptr(), wsb, None))
    out["wgrad"] = relerr(host(DW).reshape(wt.shape), ref_dw)
    if cfg is not None:
        for op in (0, 2):
            ffi.check("reset", L.jr_conv2d_set_config(ctypes.byref(d), op, X8P, 0, -1))
        if cin % 8 == 0:
            for ph in range(s * s):
                ffi.check("reset", L.jr_conv2d_set_config(ctypes.byref(d), 1, X8P, ph, -1))
    return out


def _check(out, tag=""):
    assert out["fwd"] < 5e-6, (tag, out)
    if "dgrad" in out:
        assert out["dgrad"] < 5e-6 and out["dgrad_acc"] < 5e-6, (tag, out)
    assert out["wgrad"] < 1e-5, (tag, out)


@pytest.mark.parametrize("case", CASES)
def test_conv_x8p(case):
    ffi = _lib()
    _check(_run(ffi, ffi.load(), case, seed=sum(case[:8]) * 13 + 3), case)


@pytest.mark.parametrize("case", [(2, 17, 17, 64, 96, 3, 3, 1, "same"), (2, 17, 17, 48, 64, 3, 3, 2, "valid"),
                                  (2, 11, 11, 3, 32, 3, 3, 2, "valid"), (2, 8, 8, 128, 64, 1, 1, 1, "same")])
def test_conv_x8p_every_tile_config(case):
    """Every X8P tile (fast and generic kernels), planner / forced split-K 1 and 3."""
    ffi = _lib()
    L = ffi.load()
    n, h, w, cin, cout, kh, kw, s, pad = case
    extra = 3 * 4 * max(n * h * w * 8 * cout, kh * kw * 8 * cout) * 4
    for t in range(L.jr_conv2d_num_configs(X8P)):
        for sp in (0, 1, 3):
            _check(_run(ffi, L, case, seed=11, cfg=t | (sp << 8), extra_ws=extra), (t, sp))


@pytest.mark.parametrize("case", [(2, 35, 35, 192, 64, 1, 1, 1, "same"), (2, 17, 17, 160, 160, 7, 1, 1, "same"),
                                  (2, 35, 35, 288, 384, 3, 3, 2, "valid"), (2, 8, 8, 448, 384, 3, 3, 1, "same")])
def test_x8p_bitwise_equals_x8(case):
    """Same tile geometry (128x128, BK 16) and one split: X8P reproduces the
    in-register-split X8 kernel bit for bit, for fwd, every dgrad phase and
    wgrad."""
    ffi = _lib()
    L = ffi.load()
    n, h, w, cin, cout, kh, kw, s, pad = case
    rng = np.random.default_rng(17)
    x = rng.standard_normal((n, h, w, cin)).astype(np.float32)
    wt = (rng.standard_normal((kh, kw, cin, cout)) / np.sqrt(kh * kw * cin)).astype(np.float32)
    d, ho, wo = _desc(ffi, n, h, w, cin, cout, kh, kw, s, pad)
    dy = rng.standard_normal((n, ho, wo, cout)).astype(np.float32)
    X, DY = dev(x), dev(dy)
    W, HW, WT = weight_planes(ffi, L, wt)
    XP, DYP = split_planes(ffi, L, x.reshape(-1, cin)), split_planes(ffi, L, dy.reshape(-1, cout))
    cfg = 0 | (1 << 8)
    for dt in (X8, X8P):
        for op in (0, 2):
            ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), op, dt, 0, cfg))
        for ph in range(s * s):
            ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), 1, dt, ph, cfg))
    wsb = max(L.jr_conv2d_workspace_size(ctypes.byref(d), op, dt) for op in range(3) for dt in (X8, X8P))
    ws = zeros(wsb // 4 + 4)
    res = {}
    for dt, xa, wf, wd, dya in ((X8, X, W, W, DY), (X8P, XP, WT, HW, DYP)):
        Y, DX, DW = zeros(n * ho * wo * cout), zeros(x.size), zeros(wt.size)
        ffi.check("fwd", L.jr_conv2d_fwd(ctypes.byref(d), dt, xa.data_ptr(), wf.data_ptr(), Y.data_ptr(),
                                         ws.data_ptr(), wsb, None))
        ffi.check("dgrad", L.jr_conv2d_bwd_data(ctypes.byref(d), dt, dya.data_ptr(), wd.data_ptr(), DX.data_ptr(), 0,
                                                ws.data_ptr(), wsb, None))
        ffi.check("wgrad", L.jr_conv2d_bwd_filter(ctypes.byref(d), dt, xa.data_ptr(), dya.data_ptr(), DW.data_ptr(),
                                                  ws.data_ptr(), wsb, None))
        res[dt] = (host(Y), host(DX), host(DW))
    for dt in (X8, X8P):
        for op in (0, 2):
            ffi.check("reset", L.jr_conv2d_set_config(ctypes.byref(d), op, dt, 0, -1))
        for ph in range(s * s):
            ffi.check("reset", L.jr_conv2d_set_config(ctypes.byref(d), 1, dt, ph, -1))
    for name, a, b in zip(("fwd", "dgrad", "wgrad"), res[X8], res[X8P]):
        assert np.array_equal(a, b), (name, float(np.max(np.abs(a - b))))
