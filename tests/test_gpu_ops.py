"""Per-op parity: libjr HIP kernels (through the C-ABI) vs the numpy fp64
oracle (oracle/tf_ops.py) on seeded inputs.  fp32 tolerances are stated per
test; integer/index work (argmax routing) is compared exactly."""
import ctypes

import numpy as np
import pytest

from oracle import tf_ops as R

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _lib():
    from jr import _ffi
    _ffi.init(0)
    return _ffi


_KEEP = []


@pytest.fixture(autouse=True)
def _keep_alive():
    """Device copies made by dev() live until the test ends: a temporary whose
    data_ptr() is passed to a kernel must not return to the caching allocator
    (and be handed to the next allocation) before the kernel has run."""
    yield
    torch.cuda.synchronize()
    _KEEP.clear()


def dev(a, dtype=torch.float32):
    t = torch.as_tensor(np.ascontiguousarray(a)).to("cuda", dtype=dtype)
    _KEEP.append(t)
    return t


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def relerr(got, ref):
    ref = np.asarray(ref, np.float64)
    return float(np.max(np.abs(got - ref)) / max(np.max(np.abs(ref)), 1e-30))


CONV_CASES = [
    # n, h, w, cin, cout, kh, kw, stride, padding
    (2, 35, 35, 192, 64, 1, 1, 1, "same"),
    (2, 35, 35, 48, 64, 5, 5, 1, "same"),
    (2, 17, 17, 128, 192, 1, 7, 1, "same"),
    (2, 17, 17, 160, 160, 7, 1, 1, "same"),
    (2, 35, 35, 288, 384, 3, 3, 2, "valid"),
    (3, 17, 17, 192, 320, 3, 3, 2, "valid"),
    (2, 8, 8, 448, 384, 3, 3, 1, "same"),
    (2, 8, 8, 384, 384, 1, 3, 1, "same"),
    (2, 73, 73, 80, 192, 3, 3, 1, "valid"),
    (2, 37, 37, 3, 32, 3, 3, 2, "valid"),     # conv1 (scalar A path)
    (1, 29, 31, 32, 48, 3, 3, 1, "same"),     # ragged M / N tails
]


def _desc(ffi, n, h, w, cin, cout, kh, kw, s, pad, x_off=0, x_stride=None, y_off=0, y_stride=None):
    ph, pw = ((kh - 1) // 2, (kw - 1) // 2) if pad == "same" else (0, 0)
    ho, wo = (h + 2 * ph - kh) // s + 1, (w + 2 * pw - kw) // s + 1
    return ffi.ConvDesc(n, h, w, cin, cout, kh, kw, s, s, ph, pw, ho, wo, x_off, x_stride or cin,
                        y_off, y_stride or cout), ho, wo


def _ws(ffi, d, op, dt=0):
    b = ffi.load().jr_conv2d_workspace_size(ctypes.byref(d), op, dt)
    return torch.zeros(max(b // 4, 1) + 4, device="cuda"), b


# conv dtype codes: 0 = JR_F32 (fp32 MFMA), 2 = JR_F32_X8 (fp32 tensors, products
# from the exact three-way bf16 split) -- held to the SAME fp32 tolerances
CONV_DT = [pytest.param(0, id="f32"), pytest.param(2, id="f32x8")]


@pytest.mark.parametrize("dt", CONV_DT)
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(case, dt):
    ffi = _lib()
    L = ffi.load()
    n, h, w, cin, cout, kh, kw, s, pad = case
    rng = np.random.default_rng(hash(case) % 2**31)
    x = rng.standard_normal((n, h, w, cin)).astype(np.float32)
    wt = (rng.standard_normal((kh, kw, cin, cout)) / np.sqrt(kh * kw * cin)).astype(np.float32)
    cs = (cin + 3) // 4 * 4          # c_in % 4 != 0: input kept 4-aligned, zero padded
    d, ho, wo = _desc(ffi, n, h, w, cin, cout, kh, kw, s, pad, x_stride=cs)
    ref = R.conv2d(x, wt, s, pad)
    xp = np.zeros((n, h, w, cs), np.float32)
    xp[..., :cin] = x
    X, W = dev(xp), dev(wt)
    Y = torch.zeros(n * ho * wo * cout, device="cuda")
    ws, wsb = _ws(ffi, d, 0, dt)
    ffi.check("fwd", L.jr_conv2d_fwd(ctypes.byref(d), dt, X.data_ptr(), W.data_ptr(), Y.data_ptr(),
                                     ws.data_ptr(), wsb, None))
    got = host(Y).reshape(ref.shape)
    assert relerr(got, ref) < 5e-6, relerr(got, ref)

    dy = rng.standard_normal(ref.shape).astype(np.float32)
    DY = dev(dy)
    if cin % 4 == 0 and cout % 16 == 0:
        ref_dx = R.conv2d_bwd_data(dy, wt, x.shape, s, pad)
        DX = torch.zeros(x.size, device="cuda")
        ws, wsb = _ws(ffi, d, 1, dt)
        ffi.check("dgrad", L.jr_conv2d_bwd_data(ctypes.byref(d), dt, DY.data_ptr(), W.data_ptr(), DX.data_ptr(),
                                                0, ws.data_ptr(), wsb, None))
        got = host(DX).reshape(x.shape)
        assert relerr(got, ref_dx) < 5e-6, relerr(got, ref_dx)
        # accumulate = 1 adds into the existing gradient
        ffi.check("dgrad acc", L.jr_conv2d_bwd_data(ctypes.byref(d), dt, DY.data_ptr(), W.data_ptr(),
                                                    DX.data_ptr(), 1, ws.data_ptr(), wsb, None))
        got = host(DX).reshape(x.shape)
        assert relerr(got, 2 * ref_dx) < 5e-6
    ref_dw = R.conv2d_bwd_filter(x, dy, wt.shape, s, pad)
    DW = torch.zeros(wt.size, device="cuda")
    ws, wsb = _ws(ffi, d, 2, dt)
    ffi.check("wgrad", L.jr_conv2d_bwd_filter(ctypes.byref(d), dt, X.data_ptr(), DY.data_ptr(), DW.data_ptr(),
                                              ws.data_ptr(), wsb, None))
    got = host(DW).reshape(wt.shape)
    assert relerr(got, ref_dw) < 1e-5, relerr(got, ref_dw)


@pytest.mark.parametrize("dt", CONV_DT)
@pytest.mark.parametrize("case", [(2, 17, 17, 64, 96, 3, 3, 1, "same"), (2, 17, 17, 48, 64, 3, 3, 2, "valid"),
                                  (2, 11, 11, 3, 32, 3, 3, 2, "valid")])
def test_conv_every_tile_config(case, dt):
    """Every tile configuration the autotuner may pick is correct, with the
    planner's split-K factor and with forced factors (id = tile | splits << 8)."""
    ffi = _lib()
    L = ffi.load()
    n, h, w, cin, cout, kh, kw, s, pad = case
    rng = np.random.default_rng(7)
    x = rng.standard_normal((n, h, w, cin)).astype(np.float32)
    wt = (rng.standard_normal((kh, kw, cin, cout)) / np.sqrt(kh * kw * cin)).astype(np.float32)
    cs = (cin + 3) // 4 * 4
    xp = np.zeros((n, h, w, cs), np.float32)
    xp[..., :cin] = x
    d, ho, wo = _desc(ffi, n, h, w, cin, cout, kh, kw, s, pad, x_stride=cs)
    ref = R.conv2d(x, wt, s, pad)
    dy = rng.standard_normal(ref.shape).astype(np.float32)
    ref_dx = R.conv2d_bwd_data(dy, wt, x.shape, s, pad) if cin % 4 == 0 else None
    ref_dw = R.conv2d_bwd_filter(x, dy, wt.shape, s, pad)
    X, W, DY = dev(xp), dev(wt), dev(dy)
    wsb = max(L.jr_conv2d_workspace_size(ctypes.byref(d), op, dt) for op in range(3))
    wsb += 3 * 4 * max(n * ho * wo * cout, kh * kw * cs * cout, n * h * w * cs)   # forced splits of 3
    ws = torch.zeros(wsb // 4 + 4, device="cuda")
    cfgs = [t | (sp << 8) for t in range(L.jr_conv2d_num_configs(dt)) for sp in (0, 1, 3)]  # forced split-K
    for cfg in cfgs:
        ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), 0, dt, 0, cfg))
        ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), 2, dt, 0, cfg))
        Y = torch.zeros(ref.size, device="cuda")
        ffi.check("fwd", L.jr_conv2d_fwd(ctypes.byref(d), dt, X.data_ptr(), W.data_ptr(), Y.data_ptr(),
                                         ws.data_ptr(), wsb, None))
        assert relerr(host(Y).reshape(ref.shape), ref) < 5e-6, cfg
        DW = torch.zeros(wt.size, device="cuda")
        ffi.check("wgrad", L.jr_conv2d_bwd_filter(ctypes.byref(d), dt, X.data_ptr(), DY.data_ptr(), DW.data_ptr(),
                                                  ws.data_ptr(), wsb, None))
        assert relerr(host(DW).reshape(wt.shape), ref_dw) < 1e-5, cfg
        if ref_dx is not None:
            for ph in range(s * s):
                ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), 1, dt, ph, cfg))
            DX = torch.zeros(x.size, device="cuda")
            ffi.check("dgrad", L.jr_conv2d_bwd_data(ctypes.byref(d), dt, DY.data_ptr(), W.data_ptr(), DX.data_ptr(),
                                                    0, ws.data_ptr(), wsb, None))
            assert relerr(host(DX).reshape(x.shape), ref_dx) < 5e-6, cfg
    for op in (0, 2):                    # drop the overrides: later tests get the planner's choice
        ffi.check("reset", L.jr_conv2d_set_config(ctypes.byref(d), op, dt, 0, -1))
    if ref_dx is not None:
        for ph in range(s * s):
            ffi.check("reset", L.jr_conv2d_set_config(ctypes.byref(d), 1, dt, ph, -1))


@pytest.mark.parametrize("case", [(4, 8, 8, 2048, 384, 1, 1, 1, "same"), (4, 17, 17, 192, 192, 7, 1, 1, "same"),
                                  (2, 35, 35, 288, 384, 3, 3, 2, "valid")])
def test_conv_x8_error_matches_fp32(case):
    """JR_F32_X8 is fp32 arithmetic, not reduced precision: on long
    reductions (K up to 2,592) its max error against the fp64 oracle stays
    within 2x the native fp32-MFMA kernel's, for fwd, dgrad and wgrad."""
    ffi = _lib()
    L = ffi.load()
    n, h, w, cin, cout, kh, kw, s, pad = case
    rng = np.random.default_rng(11)
    x = rng.standard_normal((n, h, w, cin)).astype(np.float32)
    wt = (rng.standard_normal((kh, kw, cin, cout)) / np.sqrt(kh * kw * cin)).astype(np.float32)
    d, ho, wo = _desc(ffi, n, h, w, cin, cout, kh, kw, s, pad)
    ref = R.conv2d(x, wt, s, pad)
    dy = rng.standard_normal(ref.shape).astype(np.float32)
    ref_dx = R.conv2d_bwd_data(dy, wt, x.shape, s, pad)
    ref_dw = R.conv2d_bwd_filter(x, dy, wt.shape, s, pad)
    X, W, DY = dev(x), dev(wt), dev(dy)
    err = {}
    for dt in (0, 2):
        Y = torch.zeros(ref.size, device="cuda")
        DX = torch.zeros(x.size, device="cuda")
        DW = torch.zeros(wt.size, device="cuda")
        ws, wsb = _ws(ffi, d, 0, dt)
        ffi.check("fwd", L.jr_conv2d_fwd(ctypes.byref(d), dt, X.data_ptr(), W.data_ptr(), Y.data_ptr(),
                                         ws.data_ptr(), wsb, None))
        ws, wsb = _ws(ffi, d, 1, dt)
        ffi.check("dgrad", L.jr_conv2d_bwd_data(ctypes.byref(d), dt, DY.data_ptr(), W.data_ptr(), DX.data_ptr(),
                                                0, ws.data_ptr(), wsb, None))
        ws, wsb = _ws(ffi, d, 2, dt)
        ffi.check("wgrad", L.jr_conv2d_bwd_filter(ctypes.byref(d), dt, X.data_ptr(), DY.data_ptr(), DW.data_ptr(),
                                                  ws.data_ptr(), wsb, None))
        err[dt] = (relerr(host(Y).reshape(ref.shape), ref), relerr(host(DX).reshape(x.shape), ref_dx),
                   relerr(host(DW).reshape(wt.shape), ref_dw))
    for e32, ex8 in zip(err[0], err[2]):
        assert ex8 <= 2.0 * e32 + 2e-7, err


def test_conv_channel_slices():
    """Input read from / output written to channel slices of wider buffers
    (concat-free Inception-block writes)."""
    ffi = _lib()
    L = ffi.load()
    n, h, w, cin, cout = 2, 9, 9, 32, 48
    rng = np.random.default_rng(5)
    big_x = rng.standard_normal((n, h, w, 80)).astype(np.float32)
    x = big_x[..., 16:48]
    wt = rng.standard_normal((3, 3, cin, cout)).astype(np.float32) * 0.1
    d, ho, wo = _desc(ffi, n, h, w, cin, cout, 3, 3, 1, "same", x_off=16, x_stride=80, y_off=64, y_stride=128)
    ref = R.conv2d(x, wt, 1, "same")
    Y = torch.full((n * ho * wo * 128,), 7.0, device="cuda")
    ws, wsb = _ws(ffi, d, 0)
    ffi.check("fwd", L.jr_conv2d_fwd(ctypes.byref(d), 0, dev(big_x).data_ptr(), dev(wt).data_ptr(), Y.data_ptr(),
                                     ws.data_ptr(), wsb, None))
    got = host(Y).reshape(n, ho, wo, 128)
    assert relerr(got[..., 64:112], ref) < 2e-6
    assert np.all(got[..., :64] == 7.0) and np.all(got[..., 112:] == 7.0)


def test_conv_rejects_bad_geometry():
    ffi = _lib()
    L = ffi.load()
    d, _, _ = _desc(ffi, 1, 8, 8, 16, 16, 3, 3, 1, "same")
    d.ho = 9
    rc = L.jr_conv2d_fwd(ctypes.byref(d), 0, 1, 1, 1, None, 0, None)
    assert rc == -1 and "ho/wo" in ffi.last_error()


@pytest.mark.parametrize("m,c", [(2 * 35 * 35, 64), (3 * 17 * 17, 192), (64 * 8 * 8, 448), (5, 48), (100003, 80)])
def test_bn_relu_fwd_bwd(m, c):
    ffi = _lib()
    L = ffi.load()
    rng = np.random.default_rng(m + c)
    x = (rng.standard_normal((m, c)) * 3 + rng.standard_normal(c) * 2).astype(np.float32)
    beta = (rng.standard_normal(c) * 0.5).astype(np.float32)
    dy = rng.standard_normal((m, c)).astype(np.float32)
    y_ref, mean_ref, inv_ref = R.bn_relu_fwd(x, beta)
    X, BETA = dev(x), dev(beta)
    MEAN, INV = torch.zeros(c, device="cuda"), torch.zeros(c, device="cuda")
    wsb = L.jr_bn_workspace_size(m, c)
    ws = torch.zeros(wsb // 4 + 4, device="cuda")
    ffi.check("stats", L.jr_bn_stats(0, X.data_ptr(), m, c, 1e-3, MEAN.data_ptr(), INV.data_ptr(),
                                     ws.data_ptr(), wsb, None))
    assert relerr(host(MEAN), mean_ref) < 1e-6
    assert relerr(host(INV), inv_ref) < 1e-6
    # read x as channel slice [4, 4 + c) of a wider raw buffer (a fused
    # sibling-conv group) and write into a channel slice of a wider output
    XW = np.zeros((m, c + 12), np.float32)
    XW[:, 4:4 + c] = x
    XS = dev(XW)
    Y = torch.zeros(m * (c + 16), device="cuda")
    ffi.check("apply", L.jr_bn_relu_apply(0, XS.data_ptr(), 4, c + 12, m, c, MEAN.data_ptr(), INV.data_ptr(),
                                          BETA.data_ptr(), Y.data_ptr(), 16, c + 16, None))
    got = host(Y).reshape(m, c + 16)
    assert np.max(np.abs(got[:, 16:] - y_ref)) < 2e-5 * max(1.0, np.abs(y_ref).max())
    assert np.all(got[:, :16] == 0)
    dx_ref, db_ref = R.bn_relu_bwd(dy, x, beta, mask=got[:, 16:] > 0)
    DYb = np.zeros((m, c + 8), np.float32)
    DYb[:, 8:] = dy
    DX, DB = torch.full((m * (c + 12),), 7.0, device="cuda"), torch.zeros(c, device="cuda")
    ffi.check("bwd", L.jr_bn_relu_bwd(0, dev(DYb).data_ptr(), 8, c + 8, XS.data_ptr(), 4, c + 12, m, c,
                                      MEAN.data_ptr(), INV.data_ptr(), BETA.data_ptr(), DX.data_ptr(), DB.data_ptr(),
                                      ws.data_ptr(), wsb, None))
    dxg = host(DX).reshape(m, c + 12)
    assert np.all(dxg[:, :4] == 7.0) and np.all(dxg[:, 4 + c:] == 7.0)   # only the slice is written
    assert relerr(host(DB), db_ref) < 1e-5
    assert relerr(dxg[:, 4:4 + c], dx_ref) < 1e-4


@pytest.mark.parametrize("shape", [(2, 147, 147, 64), (2, 35, 35, 288), (3, 17, 17, 768), (1, 9, 10, 8)])
def test_maxpool(shape):
    ffi = _lib()
    L = ffi.load()
    n, h, w, c = shape
    rng = np.random.default_rng(sum(shape))
    x = np.maximum(rng.standard_normal(shape), 0).astype(np.float32)   # post-ReLU input (ties at 0)
    y_ref, am_ref = R.maxpool3x3s2(x)
    ho, wo = y_ref.shape[1:3]
    d = ffi.PoolDesc(n, h, w, c, ho, wo, 0, c, 0, c)
    X = dev(x)
    Y = torch.zeros(y_ref.size, device="cuda")
    AM = torch.zeros(y_ref.size, dtype=torch.uint8, device="cuda")
    ffi.check("mp fwd", L.jr_maxpool3x3s2_fwd(ctypes.byref(d), 0, X.data_ptr(), Y.data_ptr(), AM.data_ptr(), None))
    assert np.array_equal(host(Y).reshape(y_ref.shape), y_ref.astype(np.float32))
    assert np.array_equal(host(AM).reshape(y_ref.shape), am_ref)
    dy = rng.standard_normal(y_ref.shape).astype(np.float32)
    dx_ref = R.maxpool3x3s2_bwd(dy, am_ref, x.shape)
    DX = torch.ones(x.size, device="cuda")
    ffi.check("mp bwd", L.jr_maxpool3x3s2_bwd(ctypes.byref(d), 0, AM.data_ptr(), dev(dy).data_ptr(), DX.data_ptr(),
                                              1, None))
    assert np.allclose(host(DX).reshape(x.shape), dx_ref + 1.0, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("shape", [(2, 35, 35, 192), (2, 17, 17, 768), (2, 8, 8, 1280), (1, 3, 5, 4)])
def test_avgpool(shape):
    ffi = _lib()
    L = ffi.load()
    n, h, w, c = shape
    rng = np.random.default_rng(sum(shape) + 1)
    x = rng.standard_normal(shape).astype(np.float32)
    y_ref = R.avgpool3x3s1_same(x)
    d = ffi.PoolDesc(n, h, w, c, h, w, 0, c, 0, c)
    Y = torch.zeros(x.size, device="cuda")
    ffi.check("ap fwd", L.jr_avgpool3x3s1_fwd(ctypes.byref(d), 0, dev(x).data_ptr(), Y.data_ptr(), None))
    assert relerr(host(Y).reshape(shape), y_ref) < 1e-6
    dy = rng.standard_normal(shape).astype(np.float32)
    dx_ref = R.avgpool3x3s1_same_bwd(dy)
    DX = torch.zeros(x.size, device="cuda")
    ffi.check("ap bwd", L.jr_avgpool3x3s1_bwd(ctypes.byref(d), 0, dev(dy).data_ptr(), DX.data_ptr(), 0, None))
    assert relerr(host(DX).reshape(shape), dx_ref) < 1e-6


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("shape", [(2, 147, 147, 64), (2, 17, 17, 48), (1, 10, 9, 8), (1, 3, 3, 4)])
def test_pools_in_channel_slices(shape, dtype):
    """Pools reading and writing channel slices of wider NHWC buffers (the
    concat-free block layout), both dtypes, accumulate and overwrite: the
    2x2-cell max-pool backward and the sliding-box avg-pool against the oracle
    on the same (bf16-rounded) inputs; bytes outside the slices untouched."""
    ffi = _lib()
    L = ffi.load()
    n, h, w, c = shape
    td = torch.bfloat16 if dtype == "bf16" else torch.float32
    dt = 1 if dtype == "bf16" else 0
    tol = 2.0 ** -7 if dtype == "bf16" else 1e-6
    rng = np.random.default_rng(sum(shape) + 7)
    rnd = lambda a: torch.as_tensor(a).to(td).float().numpy().astype(np.float64)  # noqa: E731
    xo, xs, yo, ys = 4, c + 12, 8, c + 16
    x = rnd(np.maximum(rng.standard_normal(shape), 0))
    xbuf = np.full((n, h, w, xs), 3.0)
    xbuf[..., xo:xo + c] = x
    X = dev(xbuf, td)
    y_ref, am_ref = R.maxpool3x3s2(x)
    ho, wo = y_ref.shape[1:3]
    d = ffi.PoolDesc(n, h, w, c, ho, wo, xo, xs, yo, ys)
    Y = torch.full((n * ho * wo * ys,), 5.0, device="cuda", dtype=td)
    AM = torch.zeros(n * ho * wo * c, dtype=torch.uint8, device="cuda")
    ffi.check("mp fwd", L.jr_maxpool3x3s2_fwd(ctypes.byref(d), dt, X.data_ptr(), Y.data_ptr(), AM.data_ptr(), None))
    yg = host(Y.float()).reshape(n, ho, wo, ys)
    assert np.array_equal(yg[..., yo:yo + c], y_ref) and np.all(yg[..., :yo] == 5) and np.all(yg[..., yo + c:] == 5)
    assert np.array_equal(host(AM).reshape(n, ho, wo, c), am_ref)
    dy = rnd(rng.standard_normal(y_ref.shape))
    dybuf = np.zeros((n, ho, wo, ys))
    dybuf[..., yo:yo + c] = dy
    dx_ref = R.maxpool3x3s2_bwd(dy, am_ref, x.shape)
    for acc in (0, 1):
        DX = dev(np.full((n, h, w, xs), 2.0), td)
        ffi.check("mp bwd", L.jr_maxpool3x3s2_bwd(ctypes.byref(d), dt, AM.data_ptr(), dev(dybuf, td).data_ptr(),
                                                  DX.data_ptr(), acc, None))
        g = host(DX.float()).reshape(n, h, w, xs)
        assert np.all(g[..., :xo] == 2) and np.all(g[..., xo + c:] == 2)
        assert relerr(g[..., xo:xo + c], dx_ref + 2.0 * acc) <= tol
    da = ffi.PoolDesc(n, h, w, c, h, w, xo, xs, yo, ys)
    Ya = torch.full((n * h * w * ys,), 5.0, device="cuda", dtype=td)
    ffi.check("ap fwd", L.jr_avgpool3x3s1_fwd(ctypes.byref(da), dt, X.data_ptr(), Ya.data_ptr(), None))
    ya = host(Ya.float()).reshape(n, h, w, ys)
    assert relerr(ya[..., yo:yo + c], R.avgpool3x3s1_same(x)) <= tol and np.all(ya[..., :yo] == 5)
    dya = np.zeros((n, h, w, ys))
    dya[..., yo:yo + c] = rnd(rng.standard_normal((n, h, w, c)))
    DXa = dev(np.full((n, h, w, xs), 2.0), td)
    ffi.check("ap bwd", L.jr_avgpool3x3s1_bwd(ctypes.byref(da), dt, dev(dya, td).data_ptr(), DXa.data_ptr(), 1, None))
    ga = host(DXa.float()).reshape(n, h, w, xs)
    assert relerr(ga[..., xo:xo + c], R.avgpool3x3s1_same_bwd(dya[..., yo:yo + c]) + 2.0) <= tol
    assert np.all(ga[..., :xo] == 2) and np.all(ga[..., xo + c:] == 2)


def test_gap_head_loss():
    ffi = _lib()
    L = ffi.load()
    rng = np.random.default_rng(11)
    n, hw, c = 5, 64, 2048
    x = np.maximum(rng.standard_normal((n, hw, c)), 0).astype(np.float32)
    W = (rng.standard_normal((c, 1)) * 0.05).astype(np.float32)
    b = np.array([0.1], np.float32)
    y = np.array([[0], [1], [1], [0], [1]], np.float32)
    F = torch.zeros(n * c, device="cuda")
    ffi.check("gap", L.jr_gap_fwd(0, dev(x).data_ptr(), n, hw, c, F.data_ptr(), None))
    f_ref = R.global_avg_pool(x.reshape(n, 8, 8, c))
    assert relerr(host(F).reshape(n, c), f_ref) < 1e-6
    LOG, PR, LOSS = (torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda"), torch.zeros(1, device="cuda"))
    Wd, Y = dev(W), dev(y)
    ffi.check("head", L.jr_head_fwd(0, F.data_ptr(), Wd.data_ptr(), dev(b).data_ptr(), Y.data_ptr(), n, c, 1,
                                    LOG.data_ptr(), PR.data_ptr(), LOSS.data_ptr(), None))
    z_ref = R.dense(f_ref, W, b)
    assert relerr(host(LOG).reshape(n, 1), z_ref) < 1e-5
    assert np.allclose(host(PR).reshape(n, 1), R.sigmoid(z_ref), atol=1e-6)
    assert abs(host(LOSS)[0] - R.sigmoid_xent_mean(z_ref, y)) < 1e-6
    DF, DW, DB = torch.zeros(n * c, device="cuda"), torch.zeros(c, device="cuda"), torch.zeros(1, device="cuda")
    ffi.check("head bwd", L.jr_head_bwd(0, F.data_ptr(), Wd.data_ptr(), PR.data_ptr(), Y.data_ptr(), n, c, 1,
                                        DF.data_ptr(), DW.data_ptr(), DB.data_ptr(), None))
    dz = R.sigmoid_xent_grad(z_ref, y)
    assert relerr(host(DW).reshape(c, 1), f_ref.T @ dz) < 1e-5
    assert relerr(host(DB), dz.sum(0)) < 1e-5
    assert relerr(host(DF).reshape(n, c), dz @ W.T) < 1e-5
    DX = torch.zeros(n * hw * c, device="cuda")
    ffi.check("gap bwd", L.jr_gap_bwd(0, DF.data_ptr(), n, hw, c, DX.data_ptr(), None))
    assert relerr(host(DX).reshape(n, hw, c), np.repeat((dz @ W.T)[:, None, :] / hw, hw, axis=1)) < 1e-5


def test_optimizers():
    ffi = _lib()
    L = ffi.load()
    rng = np.random.default_rng(3)
    n = 1003
    w, g, a = (rng.standard_normal(n).astype(np.float32) for _ in range(3))
    W, G, A = dev(w), dev(g), dev(a)
    ffi.check("nest", L.jr_nesterov_update(W.data_ptr(), G.data_ptr(), A.data_ptr(), n, 3e-3, 0.9, 1.0, None))
    w_ref, a_ref = R.nesterov(w.astype(np.float64), g, a, 3e-3, 0.9)
    assert np.allclose(host(W), w_ref, rtol=1e-6, atol=1e-7)
    assert np.allclose(host(A), a_ref, rtol=1e-6, atol=1e-7)
    W2 = dev(w)
    ffi.check("sgd", L.jr_sgd_update(W2.data_ptr(), G.data_ptr(), n, 3e-3, 1.0, None))
    assert np.allclose(host(W2), R.sgd(w.astype(np.float64), g, 3e-3), rtol=1e-6, atol=1e-7)


def test_u8_scale_is_tf_convert_image_dtype():
    ffi = _lib()
    L = ffi.load()
    u8 = np.arange(256, dtype=np.uint8)
    out = torch.zeros(256, device="cuda")
    ffi.check("u8", L.jr_u8_to_f32_scaled(dev(u8, torch.uint8).data_ptr(), out.data_ptr(), 0, 256, None))
    assert np.array_equal(host(out), R.convert_image_dtype_u8(u8))


@pytest.mark.parametrize("dt", [0, 1], ids=["f32", "bf16"])
def test_bn_relu_bwd_multi_segments(dt):
    """jr_bn_relu_bwd_multi: one backward launch set for the members of a
    fused sibling launch (raw output [m][48+64+96], each member's upstream
    gradient a slice of its own wider buffer, its own beta / dbeta) equals
    the three per-member jr_bn_relu_bwd calls (the fp64 partial grouping
    differs with the channel count: within 1e-6 fp32 / one bf16 ulp) and, in
    fp32, the fp64 oracle."""
    ffi = _lib()
    L = ffi.load()
    m, cs = 64 * 17 * 17, (48, 64, 96)
    c = sum(cs)
    tdt = torch.float32 if dt == 0 else torch.bfloat16
    rng = np.random.default_rng(11)
    x = (rng.standard_normal((m, c)) * 2 + rng.standard_normal(c)).astype(np.float32)
    X = torch.as_tensor(x).to(tdt).cuda()
    xs = X.float()
    MEAN = xs.double().mean(0).float()
    INV = (1.0 / torch.sqrt(xs.double().var(0, unbiased=False) + 1e-3)).float()
    dys, betas, offs, strides = [], [], (8, 0, 16), (cs[0] + 16, cs[1], cs[2] + 24)
    for k, ck in enumerate(cs):
        buf = torch.zeros((m, strides[k]), dtype=tdt, device="cuda")
        buf[:, offs[k]:offs[k] + ck] = torch.as_tensor(rng.standard_normal((m, ck)).astype(np.float32)).to(tdt)
        dys.append(buf)
        betas.append(torch.as_tensor((rng.standard_normal(ck) * 0.5).astype(np.float32)).cuda())
    wsb = L.jr_bn_workspace_size(m, c)
    ws = torch.zeros(wsb // 4 + 4, device="cuda")
    DB = [torch.zeros(ck, device="cuda") for ck in cs]
    DX = torch.full((m, c), 7.0, dtype=tdt, device="cuda")
    segs = (ffi.BnSeg * 3)(*[ffi.BnSeg(dys[k].data_ptr(), offs[k], strides[k], cs[k], betas[k].data_ptr(),
                                       DB[k].data_ptr()) for k in range(3)])
    ffi.check("multi", L.jr_bn_relu_bwd_multi(dt, 3, ctypes.byref(segs), X.data_ptr(), 0, c, m, c,
                                               MEAN.data_ptr(), INV.data_ptr(), DX.data_ptr(), ws.data_ptr(), wsb,
                                               None))
    # per member: the member's slice of x / dx / mean / invstd
    DX1 = torch.full((m, c), 7.0, dtype=tdt, device="cuda")
    DB1 = [torch.zeros(ck, device="cuda") for ck in cs]
    c0 = 0
    esz = 4 if dt == 0 else 2
    for k, ck in enumerate(cs):
        ffi.check("single", L.jr_bn_relu_bwd(dt, dys[k].data_ptr(), offs[k], strides[k], X.data_ptr(), c0, c, m, ck,
                                              MEAN.data_ptr() + 4 * c0, INV.data_ptr() + 4 * c0,
                                              betas[k].data_ptr(), DX1.data_ptr(), DB1[k].data_ptr(),
                                              ws.data_ptr(), wsb, None))
        c0 += ck
    torch.cuda.synchronize()
    d0, d1 = DX1.float().cpu().numpy(), DX.float().cpu().numpy()
    for k in range(3):
        assert relerr(DB[k].cpu().numpy(), DB1[k].cpu().numpy()) <= 1e-6
    if dt == 0:
        assert relerr(d1, d0) <= 1e-6
        beta = np.concatenate([b.cpu().numpy() for b in betas])
        dy = np.concatenate([dys[k][:, offs[k]:offs[k] + cs[k]].cpu().numpy() for k in range(3)], axis=1)
        pre = (x - MEAN.cpu().numpy()) * INV.cpu().numpy() + beta
        dx_ref, db_ref = R.bn_relu_bwd(dy, x, beta, mask=pre > 0)
        assert relerr(d1, dx_ref) < 1e-4
        assert relerr(np.concatenate([b.cpu().numpy() for b in DB]), db_ref) < 1e-5
    else:
        # bf16 sums each thread's batch of rows in fp32 before the fp64
        # combine, and which rows form a batch depends on the channel count:
        # the two k1 = mean(dy'), k2 = mean(dy' xhat) differ at fp32 rounding
        # (~1e-7 of the terms), which dx = invstd (dy' - k1 - xhat k2) can
        # expose where it cancels.  Bar: one bf16 ulp of dx, plus 1e-5 of the
        # expression's term scale (an indexing or segment bug is O(1) of it).
        beta = np.concatenate([b.cpu().numpy() for b in betas])
        dy = np.concatenate([dys[k][:, offs[k]:offs[k] + cs[k]].float().cpu().numpy() for k in range(3)], axis=1)
        xf = X.float().cpu().numpy()
        xh = (xf - MEAN.cpu().numpy()) * INV.cpu().numpy()
        g = np.where(xh + beta > 0, dy, 0.0)
        scale = INV.cpu().numpy() * (np.abs(g) + np.abs(g).mean(0) + np.abs(xh) * np.abs(g * xh).mean(0))
        assert np.all(np.abs(d1 - d0) <= np.abs(d0) * 2.0 ** -7 + 1e-5 * scale)
    # validation: segments must sum to c
    segs[2].c = 88
    assert L.jr_bn_relu_bwd_multi(dt, 3, ctypes.byref(segs), X.data_ptr(), 0, c, m, c, MEAN.data_ptr(),
                                  INV.data_ptr(), DX.data_ptr(), ws.data_ptr(), wsb, None) == -1
    assert "sum to c" in ffi.last_error()
