"""JR_F32_X6H (jr.h): fp32 convolutions on the fp16 matrix cores from a
power-of-two-scaled three-way fp16 split, six products -- held to the SAME
fp32 bars as JR_F32_X8 (test_gpu_ops.py: 5e-6 / 1e-5 of max |ref| per op,
every tile id including the stream-K grids and the fp32-MFMA ids), its error
on long reductions within 2x the fp32-MFMA kernel's with data gradients of
1e-7 scale (the operand scales at work), and the magnitude words that feed
the scales: jr_absmax_prep per parameter block (+ its bound guard) and the BN
backward's fused max (bitwise the plain backward's dx)."""
import ctypes

import numpy as np
import pytest

from oracle import tf_ops as R

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

X6H, F32 = 4, 0


def _lib():
    from jr import _ffi
    _ffi.init(0)
    return _ffi


def relerr(got, ref):
    ref = np.asarray(ref, np.float64)
    return float(np.max(np.abs(got - ref)) / max(np.max(np.abs(ref)), 1e-30))


def _words(v, lane=5):
    """64 magnitude words whose max is v (the rest smaller)."""
    w = torch.zeros(64, device="cuda")
    w[lane] = float(v)
    w[(lane + 7) % 64] = float(v) / 3
    return w


def _desc(ffi, n, h, w, cin, cout, kh, kw, s, pad):
    ph, pw = ((kh - 1) // 2, (kw - 1) // 2) if pad == "same" else (0, 0)
    ho, wo = (h + 2 * ph - kh) // s + 1, (w + 2 * pw - kw) // s + 1
    cs = (cin + 3) // 4 * 4
    return ffi.ConvDesc(n, h, w, cin, cout, kh, kw, s, s, ph, pw, ho, wo, 0, cs, 0, cout), ho, wo, cs


def _setup(ffi, case, seed, dy_scale=1.0):
    n, h, w, cin, cout, kh, kw, s, pad = case
    rng = np.random.default_rng(seed)
    x = np.maximum(rng.standard_normal((n, h, w, cin)), 0).astype(np.float32)     # BN + ReLU-like
    wt = (rng.standard_normal((kh, kw, cin, cout)) / np.sqrt(kh * kw * cin)).astype(np.float32)
    d, ho, wo, cs = _desc(ffi, n, h, w, cin, cout, kh, kw, s, pad)
    dy = (rng.standard_normal((n, ho, wo, cout)) * dy_scale).astype(np.float32)
    xp = np.zeros((n, h, w, cs), np.float32)
    xp[..., :cin] = x
    X, W, DY = (torch.as_tensor(a).cuda() for a in (xp, wt, dy))
    # x: a host bound (as the engine passes for activations); w, dy: device words
    wm, gm = _words(np.abs(wt).max()), _words(np.abs(dy).max())
    d.x_bound = float(x.max()) * 1.5
    d.w_absmax, d.dy_absmax = wm.data_ptr(), gm.data_ptr()
    return d, (x, wt, dy), (X, W, DY), (wm, gm)


CASES = [(2, 35, 35, 48, 64, 5, 5, 1, "same"), (2, 17, 17, 128, 192, 1, 7, 1, "same"),
         (3, 17, 17, 192, 320, 3, 3, 2, "valid"), (2, 8, 8, 448, 384, 3, 3, 1, "same"),
         (2, 73, 73, 80, 192, 3, 3, 1, "valid"), (2, 37, 37, 3, 32, 3, 3, 2, "valid"),
         (1, 29, 31, 32, 48, 3, 3, 1, "same")]


@pytest.mark.parametrize("case", CASES)
def test_x6h_fwd_dgrad_wgrad_at_fp32_bars(case):
    ffi = _lib()
    L = ffi.load()
    n, h, w, cin, cout, kh, kw, s, pad = case
    d, (x, wt, dy), (X, W, DY), keep = _setup(ffi, case, hash(case) % 2**31)
    ref = R.conv2d(x, wt, s, pad)
    wsb = max(L.jr_conv2d_workspace_size(ctypes.byref(d), op, X6H) for op in range(3))
    ws = torch.zeros(wsb // 4 + 4, device="cuda")
    Y = torch.zeros(ref.size, device="cuda")
    ffi.check("fwd", L.jr_conv2d_fwd(ctypes.byref(d), X6H, X.data_ptr(), W.data_ptr(), Y.data_ptr(), ws.data_ptr(),
                                     wsb, None))
    torch.cuda.synchronize()
    assert relerr(Y.cpu().numpy().reshape(ref.shape), ref) < 5e-6
    if cin % 4 == 0:
        ref_dx = R.conv2d_bwd_data(dy, wt, x.shape, s, pad)
        DX = torch.zeros(x.size, device="cuda")
        ffi.check("dgrad", L.jr_conv2d_bwd_data(ctypes.byref(d), X6H, DY.data_ptr(), W.data_ptr(), DX.data_ptr(), 0,
                                                ws.data_ptr(), wsb, None))
        torch.cuda.synchronize()
        assert relerr(DX.cpu().numpy().reshape(x.shape), ref_dx) < 5e-6
    ref_dw = R.conv2d_bwd_filter(x, dy, wt.shape, s, pad)
    DW = torch.zeros(wt.size, device="cuda")
    ffi.check("wgrad", L.jr_conv2d_bwd_filter(ctypes.byref(d), X6H, X.data_ptr(), DY.data_ptr(), DW.data_ptr(),
                                              ws.data_ptr(), wsb, None))
    torch.cuda.synchronize()
    assert relerr(DW.cpu().numpy().reshape(wt.shape), ref_dw) < 1e-5


@pytest.mark.parametrize("case", [(2, 17, 17, 64, 96, 3, 3, 1, "same"), (2, 17, 17, 48, 64, 3, 3, 2, "valid")])
def test_x6h_every_tile_config(case):
    """Every config id of the JR_F32_X8 id space under JR_F32_X6H (fp16
    six-product tiles, the fp32-MFMA ids, the stream-K grids), planner and
    forced split-K factors."""
    ffi = _lib()
    L = ffi.load()
    n, h, w, cin, cout, kh, kw, s, pad = case
    d, (x, wt, dy), (X, W, DY), keep = _setup(ffi, case, 7)
    ref = R.conv2d(x, wt, s, pad)
    ref_dx = R.conv2d_bwd_data(dy, wt, x.shape, s, pad)
    ref_dw = R.conv2d_bwd_filter(x, dy, wt.shape, s, pad)
    ho, wo = ref.shape[1:3]
    wsb = max(L.jr_conv2d_workspace_size(ctypes.byref(d), op, X6H) for op in range(3))
    wsb += 3 * 4 * max(n * ho * wo * cout, kh * kw * cin * cout, n * h * w * cin)
    ws = torch.zeros(wsb // 4 + 4, device="cuda")
    ncfg = L.jr_conv2d_num_configs(X6H)
    assert ncfg == L.jr_conv2d_num_configs(2)
    try:
        for cfg in [t | (sp << 8) for t in range(ncfg) for sp in (0, 3)]:
            for op in (0, 2):
                ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), op, X6H, 0, cfg))
            for ph in range(s * s):
                ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), 1, X6H, ph, cfg))
            Y, DW, DX = (torch.zeros(a.size, device="cuda") for a in (ref, wt, x))
            ffi.check("fwd", L.jr_conv2d_fwd(ctypes.byref(d), X6H, X.data_ptr(), W.data_ptr(), Y.data_ptr(),
                                             ws.data_ptr(), wsb, None))
            ffi.check("wgrad", L.jr_conv2d_bwd_filter(ctypes.byref(d), X6H, X.data_ptr(), DY.data_ptr(),
                                                      DW.data_ptr(), ws.data_ptr(), wsb, None))
            ffi.check("dgrad", L.jr_conv2d_bwd_data(ctypes.byref(d), X6H, DY.data_ptr(), W.data_ptr(), DX.data_ptr(),
                                                    0, ws.data_ptr(), wsb, None))
            torch.cuda.synchronize()
            assert relerr(Y.cpu().numpy().reshape(ref.shape), ref) < 5e-6, cfg
            assert relerr(DW.cpu().numpy().reshape(wt.shape), ref_dw) < 1e-5, cfg
            assert relerr(DX.cpu().numpy().reshape(x.shape), ref_dx) < 5e-6, cfg
        ffi.device_check()
    finally:
        for op in (0, 2):
            ffi.check("reset", L.jr_conv2d_set_config(ctypes.byref(d), op, X6H, 0, -1))
        for ph in range(s * s):
            ffi.check("reset", L.jr_conv2d_set_config(ctypes.byref(d), 1, X6H, ph, -1))


@pytest.mark.parametrize("case", [(4, 8, 8, 2048, 384, 1, 1, 1, "same"), (4, 17, 17, 192, 192, 7, 1, 1, "same"),
                                  (2, 35, 35, 288, 384, 3, 3, 2, "valid")])
def test_x6h_error_matches_fp32_tiny_gradients(case):
    """Long reductions (K up to 2,592) with data gradients of 1e-7 scale: the
    operand scales move them into fp16's range, and every op's max error vs
    fp64 stays within 2x the fp32-MFMA kernel's."""
    ffi = _lib()
    L = ffi.load()
    n, h, w, cin, cout, kh, kw, s, pad = case
    d, (x, wt, dy), (X, W, DY), keep = _setup(ffi, case, 11, dy_scale=1e-7)
    ref = R.conv2d(x, wt, s, pad)
    refs = {0: ref, 1: R.conv2d_bwd_data(dy, wt, x.shape, s, pad), 2: R.conv2d_bwd_filter(x, dy, wt.shape, s, pad)}
    err = {}
    for dt in (F32, X6H):
        wsb = max(L.jr_conv2d_workspace_size(ctypes.byref(d), op, dt) for op in range(3))
        ws = torch.zeros(wsb // 4 + 4, device="cuda")
        outs = {op: torch.zeros(refs[op].size, device="cuda") for op in range(3)}
        ffi.check("fwd", L.jr_conv2d_fwd(ctypes.byref(d), dt, X.data_ptr(), W.data_ptr(), outs[0].data_ptr(),
                                         ws.data_ptr(), wsb, None))
        ffi.check("dgrad", L.jr_conv2d_bwd_data(ctypes.byref(d), dt, DY.data_ptr(), W.data_ptr(), outs[1].data_ptr(),
                                                0, ws.data_ptr(), wsb, None))
        ffi.check("wgrad", L.jr_conv2d_bwd_filter(ctypes.byref(d), dt, X.data_ptr(), DY.data_ptr(),
                                                  outs[2].data_ptr(), ws.data_ptr(), wsb, None))
        torch.cuda.synchronize()
        err[dt] = [relerr(outs[op].cpu().numpy().reshape(refs[op].shape), refs[op]) for op in range(3)]
    print(case, "f32 mfma", err[F32], "x6h", err[X6H])
    for op in range(3):
        assert err[X6H][op] <= 2 * err[F32][op] + 1e-7, (op, err)


def test_absmax_prep_segments_and_guard():
    ffi = _lib()
    L = ffi.load()
    g = torch.Generator(device="cuda").manual_seed(3)
    src = torch.randn(300_000, device="cuda", generator=g)
    segs = [(0, 1000, 0, 0.0), (1000, 250_000, 1, 0.0), (251_000, 49_000, 2, 0.0)]
    arr = (ffi.AbsmaxSeg * 3)(*[ffi.AbsmaxSeg(*sg) for sg in segs])
    table = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).cuda()
    out = torch.full((64 * 4,), 123.0, device="cuda")
    ffi.check("prep", L.jr_absmax_prep(src.data_ptr(), table.data_ptr(), 3, out.data_ptr(), out.numel(), None))
    torch.cuda.synchronize()
    ffi.device_check()
    o = out.view(4, 64).max(1).values.cpu().numpy()
    for k, (off, cnt, row, _) in enumerate(segs):
        assert o[row] == float(src[off:off + cnt].abs().max())
    assert o[3] == 0.0                                   # zeroed, fed by no segment
    # a bound guard: the max above the limit is a device-side failure
    arr[1].limit = 0.5
    table = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).cuda()
    ffi.check("prep", L.jr_absmax_prep(src.data_ptr(), table.data_ptr(), 3, out.data_ptr(), out.numel(), None))
    torch.cuda.synchronize()
    with pytest.raises(ffi.JRError) as ei:
        ffi.device_check()
    assert ei.value.status == ffi.JR_ERR_DEVICE
    ffi.device_check()                                  # reported once, then clear


@pytest.mark.parametrize("c", [64, 192, 1024])
def test_bn_backward_absmax_is_bitwise_and_exact(c):
    """jr_bn_relu_bwd_multi_absmax: dx and dbeta bitwise jr_bn_relu_bwd_multi's,
    and the max over its 64 words is max |dx| exactly."""
    ffi = _lib()
    L = ffi.load()
    m = 64 * 17 * 17 if c <= 256 else 64 * 8 * 8
    g = torch.Generator(device="cuda").manual_seed(c)
    x = torch.randn(m * c, device="cuda", generator=g)
    dy = torch.randn(m * c, device="cuda", generator=g) * 1e-6
    beta = torch.randn(c, device="cuda", generator=g) * 0.1
    mean, var = x.view(m, c).mean(0), x.view(m, c).var(0, unbiased=False)
    invstd = torch.rsqrt(var + 1e-3)
    wsb = L.jr_bn_workspace_size(m, c)
    ws = torch.zeros(wsb // 4 + 4, device="cuda")
    outs = []
    for absmax in (False, True):
        dx = torch.zeros(m * c, device="cuda")
        db = torch.zeros(c, device="cuda")
        seg = ffi.BnSeg(dy.data_ptr(), 0, c, c, beta.data_ptr(), db.data_ptr())
        words = torch.zeros(64, device="cuda")
        args = (0, 1, ctypes.byref(seg), x.data_ptr(), 0, c, m, c, mean.data_ptr(), invstd.data_ptr(), dx.data_ptr(),
                ws.data_ptr(), wsb)
        if absmax:
            ffi.check("bwd", L.jr_bn_relu_bwd_multi_absmax(*args, words.data_ptr(), None))
        else:
            ffi.check("bwd", L.jr_bn_relu_bwd_multi(*args, None))
        torch.cuda.synchronize()
        outs.append((dx.clone(), db.clone(), words.clone()))
    (dx0, db0, _), (dx1, db1, w1) = outs
    assert torch.equal(dx0, dx1) and torch.equal(db0, db1)
    assert float(w1.max()) == float(dx1.abs().max()) > 0
