"""bf16 path parity (BASELINE configs 3 and 5): libjr bf16 kernels through the
C-ABI vs the fp64 numpy oracle evaluated on the SAME bf16-rounded inputs, so
the only error left is the kernel's: fp32 accumulation of exact bf16
products, plus one bf16 rounding of the output for FWD / DGRAD.

Tolerances (max |err| / max |ref|): FWD and DGRAD outputs are bf16, whose
rounding is <= 2^-9 relative per element -> 8e-3; WGRAD writes fp32 dW -> 1e-4.
"""
import ctypes

import numpy as np
import pytest

from oracle import tf_ops as R

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

TOL_BF16_OUT = 8e-3
TOL_F32_OUT = 1e-4

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


def bf16_round(a):
    """fp32 -> bf16 (round to nearest even, torch's cast) -> float64."""
    return torch.as_tensor(np.ascontiguousarray(a, np.float32)).to(torch.bfloat16).to(torch.float64).numpy()


def dev_bf16(a):
    t = torch.as_tensor(np.ascontiguousarray(a, np.float32)).to(torch.bfloat16).cuda()
    _KEEP.append(t)
    return t


def dev_f32(a):
    t = torch.as_tensor(np.ascontiguousarray(a, np.float32)).cuda()
    _KEEP.append(t)
    return t


def host(t):
    torch.cuda.synchronize()
    return t.to(torch.float64).cpu().numpy()


def relerr(got, ref):
    ref = np.asarray(ref, np.float64)
    return float(np.max(np.abs(got - ref)) / max(np.max(np.abs(ref)), 1e-30))


def _desc(ffi, n, h, w, cin, cout, kh, kw, s, pad, x_stride):
    ph, pw = ((kh - 1) // 2, (kw - 1) // 2) if pad == "same" else (0, 0)
    ho, wo = (h + 2 * ph - kh) // s + 1, (w + 2 * pw - kw) // s + 1
    return ffi.ConvDesc(n, h, w, cin, cout, kh, kw, s, s, ph, pw, ho, wo, 0, x_stride, 0, cout), ho, wo


def _weights(ffi, L, wt):
    """fp32 master -> (bf16 HWIO, bf16 W^T [co][kh][kw][c8]) via jr_conv_weights_bf16."""
    kh, kw, cin, cout = wt.shape
    c8 = (cin + 7) // 8 * 8
    W = dev_f32(wt)
    hwio = torch.zeros(wt.size, dtype=torch.bfloat16, device="cuda")
    wtt = torch.full((cout * kh * kw * c8,), 7.0, dtype=torch.bfloat16, device="cuda")
    _KEEP.extend([hwio, wtt])
    ffi.check("wprep", L.jr_conv_weights_bf16(W.data_ptr(), kh, kw, cin, cout, hwio.data_ptr(), wtt.data_ptr(),
                                              None))
    return hwio, wtt


def _run_all(ffi, L, case, seed, cfg=None, extra_ws=0):
    n, h, w, cin, cout, kh, kw, s, pad = case
    rng = np.random.default_rng(seed)
    x = bf16_round(rng.standard_normal((n, h, w, cin)))
    wt32 = (rng.standard_normal((kh, kw, cin, cout)) / np.sqrt(kh * kw * cin)).astype(np.float32)
    wt = bf16_round(wt32)
    c8 = (cin + 7) // 8 * 8
    d, ho, wo = _desc(ffi, n, h, w, cin, cout, kh, kw, s, pad, c8)
    xp = np.zeros((n, h, w, c8))
    xp[..., :cin] = x
    X = dev_bf16(xp)
    hwio, wtt = _weights(ffi, L, wt32)
    wsb = max(L.jr_conv2d_workspace_size(ctypes.byref(d), op, 1) for op in range(3)) + extra_ws
    ws = torch.zeros(wsb // 4 + 4, device="cuda")
    _KEEP.append(ws)
    if cfg is not None:
        for op in (0, 2):
            ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), op, 1, 0, cfg))
        if cin % 8 == 0:
            for ph in range(s * s):
                ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), 1, 1, ph, cfg))
    out = {}
    ref = R.conv2d(x, wt, s, pad)
    Y = torch.zeros(n * ho * wo * cout, dtype=torch.bfloat16, device="cuda")
    ffi.check("fwd", L.jr_conv2d_fwd(ctypes.byref(d), 1, X.data_ptr(), wtt.data_ptr(), Y.data_ptr(),
                                     ws.data_ptr(), wsb, None))
    out["fwd"] = relerr(host(Y).reshape(ref.shape), ref)
    dy = bf16_round(rng.standard_normal(ref.shape))
    DY = dev_bf16(dy)
    if cin % 8 == 0:
        ref_dx = R.conv2d_bwd_data(dy, wt, x.shape, s, pad)
        DX = torch.zeros(x.size, dtype=torch.bfloat16, device="cuda")
        ffi.check("dgrad", L.jr_conv2d_bwd_data(ctypes.byref(d), 1, DY.data_ptr(), hwio.data_ptr(), DX.data_ptr(),
                                                0, ws.data_ptr(), wsb, None))
        out["dgrad"] = relerr(host(DX).reshape(x.shape), ref_dx)
        ffi.check("dgrad acc", L.jr_conv2d_bwd_data(ctypes.byref(d), 1, DY.data_ptr(), hwio.data_ptr(),
                                                    DX.data_ptr(), 1, ws.data_ptr(), wsb, None))
        out["dgrad_acc"] = relerr(host(DX).reshape(x.shape), 2 * ref_dx)
    ref_dw = R.conv2d_bwd_filter(x, dy, wt.shape, s, pad)
    DW = torch.zeros(wt.size, device="cuda")
    ffi.check("wgrad", L.jr_conv2d_bwd_filter(ctypes.byref(d), 1, X.data_ptr(), DY.data_ptr(), DW.data_ptr(),
                                              ws.data_ptr(), wsb, None))
    out["wgrad"] = relerr(host(DW).reshape(wt.shape), ref_dw)
    return out


def _check(out):
    assert out["fwd"] < TOL_BF16_OUT, out
    if "dgrad" in out:
        assert out["dgrad"] < TOL_BF16_OUT, out
        assert out["dgrad_acc"] < 2 * TOL_BF16_OUT, out
    assert out["wgrad"] < TOL_F32_OUT, out


HALO_IDS = range(17, 25)   # jr_conv_impl.h: kNumCfgsBf16 .. + kNumHaloBf16 (the wide tiles follow)

CASES = [
    (2, 35, 35, 192, 64, 1, 1, 1, "same"),
    (2, 35, 35, 48, 64, 5, 5, 1, "same"),
    (2, 17, 17, 128, 192, 1, 7, 1, "same"),
    (2, 17, 17, 160, 160, 7, 1, 1, "same"),
    (2, 35, 35, 288, 384, 3, 3, 2, "valid"),
    (2, 8, 8, 448, 384, 3, 3, 1, "same"),
    (2, 73, 73, 80, 192, 3, 3, 1, "valid"),
    (2, 37, 37, 3, 32, 3, 3, 2, "valid"),     # conv1: c_in 3 padded to 8
    (1, 29, 31, 32, 48, 3, 3, 1, "same"),     # ragged M / N tails
]


@pytest.mark.parametrize("case", CASES)
def test_conv_bf16(case):
    ffi = _lib()
    _check(_run_all(ffi, ffi.load(), case, seed=sum(case[:8]) * 7 + 1))


@pytest.mark.parametrize("case", [(2, 17, 17, 64, 96, 3, 3, 1, "same"), (2, 17, 17, 48, 64, 3, 3, 2, "valid"),
                                  (2, 11, 11, 3, 32, 3, 3, 2, "valid"), (2, 8, 8, 128, 64, 1, 1, 1, "same")])
def test_conv_bf16_every_tile_config(case):
    """Every bf16 tile (fast and generic kernels alike), with the planner's
    split-K factor and with forced factors 1 and 3."""
    ffi = _lib()
    L = ffi.load()
    n, h, w, cin, cout, kh, kw, s, pad = case
    extra = 3 * 4 * max(n * h * w * 8 * cout, kh * kw * 8 * cout) * 4
    for t in range(L.jr_conv2d_num_configs(1)):
        for sp in (0, 1, 3):
            out = _run_all(ffi, L, case, seed=11, cfg=t | (sp << 8), extra_ws=extra)
            assert out["fwd"] < TOL_BF16_OUT and out["wgrad"] < TOL_F32_OUT, (t, sp, out)
            if "dgrad" in out:
                assert out["dgrad"] < TOL_BF16_OUT, (t, sp, out)


@pytest.mark.parametrize("case", [(2, 17, 17, 128, 192, 1, 7, 1, "same"), (2, 17, 17, 160, 160, 7, 1, 1, "same"),
                                  (2, 35, 35, 64, 96, 3, 3, 1, "same"), (2, 8, 8, 448, 384, 3, 3, 1, "same"),
                                  (2, 8, 8, 384, 384, 1, 3, 1, "same"), (2, 8, 8, 384, 384, 3, 1, 1, "same"),
                                  (1, 29, 31, 32, 48, 3, 3, 1, "same")])
def test_conv_bf16_halo_configs(case):
    """The halo-tiled forward (jr_conv_halo.hip: one halo image per 32-channel
    chunk, every tap a shifted window of it; bf16 config ids 17-24)
    against the fp64 oracle, with the planner's split-K factor and forced
    factor 2, and with the fused BN statistics.  A halo config forced on a
    geometry it does not cover falls back to the GEMM tiles (dgrad / wgrad
    here), and at least one halo config takes every case's forward."""
    ffi = _lib()
    L = ffi.load()
    n, h, w, cin, cout, kh, kw, s, pad = case
    taken = 0
    extra = 4 * 4 * n * h * w * 8 * cout
    for t in HALO_IDS:
        for sp in (0, 2):
            out = _run_all(ffi, L, case, seed=21, cfg=t | (sp << 8), extra_ws=extra)
            assert out["fwd"] < TOL_BF16_OUT and out["wgrad"] < TOL_F32_OUT, (t, sp, out)
            assert out["dgrad"] < TOL_BF16_OUT, (t, sp, out)
            d, ho, wo = _desc(ffi, n, h, w, cin, cout, kh, kw, s, pad, (cin + 7) // 8 * 8)
            taken += (L.jr_conv2d_get_config(ctypes.byref(d), 0, 1, 0) & 0xFF) == t
    assert taken > 0, case
    # fused BN statistics through the halo epilogue
    rng = np.random.default_rng(5)
    x = bf16_round(rng.standard_normal((n, h, w, cin)))
    wt32 = (rng.standard_normal((kh, kw, cin, cout)) / np.sqrt(kh * kw * cin)).astype(np.float32)
    d, ho, wo = _desc(ffi, n, h, w, cin, cout, kh, kw, s, pad, cin)
    hwio, wtt = _weights(ffi, L, wt32)
    X = dev_bf16(x)
    wsb = L.jr_conv2d_workspace_size(ctypes.byref(d), 0, 1)
    ws = torch.zeros(wsb // 4 + 4, device="cuda")
    Y = torch.zeros(n * ho * wo * cout, dtype=torch.bfloat16, device="cuda")
    MEAN, INV = torch.zeros(cout, device="cuda"), torch.zeros(cout, device="cuda")
    for t in HALO_IDS:
        ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), 0, 1, 0, t))
        if (L.jr_conv2d_get_config(ctypes.byref(d), 0, 1, 0) & 0xFF) != t:
            continue
        ffi.check("fwd+stats", L.jr_conv2d_fwd_bn_stats(ctypes.byref(d), 1, X.data_ptr(), wtt.data_ptr(), Y.data_ptr(),
                                                         ctypes.c_float(1e-3), MEAN.data_ptr(), INV.data_ptr(),
                                                         ws.data_ptr(), wsb, None))
        y = host(Y).reshape(n * ho * wo, cout).astype(np.float64)   # statistics are of y as stored
        mu = y.mean(0)
        inv = 1.0 / np.sqrt(y.var(0) + 1e-3)
        assert np.max(np.abs(MEAN.cpu().numpy() - mu)) <= 1e-5 * np.abs(y).max(), t
        assert np.max(np.abs(INV.cpu().numpy() / inv - 1)) <= 1e-5, t
    ffi.check("reset", L.jr_conv2d_set_config(ctypes.byref(d), 0, 1, 0, -1))


def test_conv_weights_bf16_layouts():
    """jr_conv_weights_bf16 and the one-launch multi-layer form write the
    bf16 HWIO copy and the zero-padded W^T [co][kh][kw][c8] exactly."""
    ffi = _lib()
    L = ffi.load()
    rng = np.random.default_rng(3)
    shapes = [(3, 3, 3, 32), (1, 7, 160, 192), (1, 1, 2048, 192), (5, 5, 48, 64)]
    ws = [rng.standard_normal(sh).astype(np.float32) for sh in shapes]
    for wt in ws:
        hwio, wtt = _weights(ffi, L, wt)
        kh, kw, cin, cout = wt.shape
        c8 = (cin + 7) // 8 * 8
        exp_t = np.zeros((cout, kh, kw, c8))
        exp_t[..., :cin] = bf16_round(wt).transpose(3, 0, 1, 2)
        assert np.array_equal(host(hwio).reshape(wt.shape), bf16_round(wt))
        assert np.array_equal(host(wtt).reshape(exp_t.shape), exp_t)
    # multi: all layers in one launch from a device table
    flat = np.concatenate([w.ravel() for w in ws])
    layers, so, ho_, to, tiles = [], 0, 0, 0, 0
    for wt in ws:
        kh, kw, cin, cout = wt.shape
        c8 = (cin + 7) // 8 * 8
        layers.append(ffi.WPrep(so, ho_, to, kh, kw, cin, cout, tiles, 0))
        tiles += L.jr_conv_weights_bf16_tiles(kh, kw, cin, cout)
        so += wt.size
        ho_ += wt.size
        to += cout * kh * kw * c8
    arr = (ffi.WPrep * len(layers))(*layers)
    tab = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).cuda()
    src = dev_f32(flat)
    hw = torch.zeros(ho_, dtype=torch.bfloat16, device="cuda")
    tt = torch.zeros(to, dtype=torch.bfloat16, device="cuda")
    _KEEP.extend([tab, hw, tt])
    ffi.check("multi", L.jr_conv_weights_bf16_multi(tab.data_ptr(), len(layers), tiles, src.data_ptr(),
                                                    hw.data_ptr(), tt.data_ptr(), None))
    assert np.array_equal(host(hw), bf16_round(flat))
    off = 0
    got_t = host(tt)
    for wt in ws:
        kh, kw, cin, cout = wt.shape
        c8 = (cin + 7) // 8 * 8
        exp_t = np.zeros((cout, kh, kw, c8))
        exp_t[..., :cin] = bf16_round(wt).transpose(3, 0, 1, 2)
        n = exp_t.size
        assert np.array_equal(got_t[off:off + n].reshape(exp_t.shape), exp_t)
        off += n
