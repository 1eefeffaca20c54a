"""BatchNormalization-backward reduce fused into the data-gradient epilogue
(jr_conv2d_bwd_data_bnp + jr_bn_relu_bwd_parts), through the C-ABI.

The ReluGrad / FusedBatchNormGrad reduction of a conv2d_bn layer (train.py:
150-153 differentiates the Keras blocks) needs sum dy' and sum dy' * xhat per
channel; when one bwd_data GEMM is the last writer of dy, its epilogue forms
them from the final values.  Checks, fp32 (x8 and fp32 MFMA) and bf16, stride
1 and the 4-phase stride-2 case, overwrite and accumulate, two slices of dx
belonging to two BN launch sets:
  * dx is BITWISE jr_conv2d_bwd_data's (the partials are a side computation);
  * the partials summed over slots equal the fp64 sums of the oracle's
    expression (oracle/tf_ops.py bn_relu_bwd terms) on dx AS STORED and the
    raw output, with jr_bn.hip's fp32 rounding of xhat and of the ReLU test:
    within 2e-5 of sum |term| (fp32 partial sums over <= 128 rows);
  * jr_bn_relu_bwd_parts equals jr_bn_relu_bwd_multi (the 3-launch path) on
    the same dy: dbeta within 2e-5 of sum |dy'|, dx within 1e-5 (fp32) /
    one bf16 ulp (bf16) of max |dx|.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

_KEEP = []


@pytest.fixture(autouse=True)
def _keep_alive():
    yield
    torch.cuda.synchronize()
    _KEEP.clear()


def _t(a, dtype):
    t = torch.as_tensor(np.ascontiguousarray(a, np.float32)).to(dtype).cuda()
    _KEEP.append(t)
    return t


def _host(t):
    return t.double().cpu().numpy()


# (n, h, w, c_in = dx channels, c_out, kh, kw, stride, padding, split of c_in)
CASES = [
    (2, 35, 35, 96, 64, 3, 3, 1, "same", 32),
    (2, 17, 17, 192, 160, 1, 7, 1, "same", 64),
    (2, 35, 35, 288, 384, 3, 3, 2, "valid", 96),    # 4 dgrad phases, one without taps on some rows
    (1, 29, 31, 48, 32, 3, 3, 1, "same", 32),        # ragged row groups, a slice ending at c_in
]


@pytest.mark.parametrize("accumulate", [0, 1])
@pytest.mark.parametrize("dtype", ["f32x8", "f32", "bf16"])
@pytest.mark.parametrize("case", CASES)
def test_dgrad_bn_partials(case, dtype, accumulate):
    from jr import _ffi
    _ffi.init(0)
    L = _ffi.load()
    dt = {"f32": 0, "bf16": 1, "f32x8": 2}[dtype]
    bdt = 1 if dtype == "bf16" else 0               # activations / BN dtype
    f32 = dtype != "bf16"
    tdt = torch.float32 if f32 else torch.bfloat16
    n, h, w, cin, cout, kh, kw, s, pad, c1 = case
    rng = np.random.default_rng(sum(case[:8]) + c1 + dt + 7 * accumulate)
    ph, pw = ((kh - 1) // 2, (kw - 1) // 2) if pad == "same" else (0, 0)
    ho, wo = (h + 2 * ph - kh) // s + 1, (w + 2 * pw - kw) // s + 1
    d = _ffi.ConvDesc(n, h, w, cin, cout, kh, kw, s, s, ph, pw, ho, wo, 0, cin, 0, cout)
    dy = _t(rng.standard_normal((n, ho, wo, cout)), tdt)
    wt = (rng.standard_normal((kh, kw, cin, cout)) / np.sqrt(kh * kw * cout)).astype(np.float32)
    if f32:
        W = _t(wt, torch.float32)
    else:
        W32 = _t(wt, torch.float32)
        W = torch.zeros(wt.size, dtype=torch.bfloat16, device="cuda")
        _KEEP.append(W)
        _ffi.check("wprep", L.jr_conv_weights_bf16(W32.data_ptr(), kh, kw, cin, cout, W.data_ptr(), None, None))
    dx0 = rng.standard_normal((n, h, w, cin))
    dx_ref, dx_bnp = _t(dx0, tdt), _t(dx0, tdt)
    # the BN layers whose ReLU outputs are dx's channel slices [0, c1) and [c1, cin):
    # raw conv output (stride cin), statistics, beta
    raw = _t(rng.standard_normal((n, h, w, cin)) * 1.5 + 0.3, tdt)
    mean = _t(rng.standard_normal(cin) * 0.3, torch.float32)
    invstd = _t(rng.random(cin) + 0.5, torch.float32)
    beta = _t(rng.standard_normal(cin) * 0.5, torch.float32)
    P = ctypes.c_int32(0)
    rc = L.jr_conv2d_bwd_data_bnp_slots(ctypes.byref(d), dt, ctypes.byref(P))
    if rc != 0:
        pytest.skip("planned dgrad splits K: " + L.jr_last_error().decode())
    P = P.value
    slices = [(0, c1), (c1, cin)]
    parts = [torch.zeros(2 * (hi - lo) * P, dtype=torch.float64, device="cuda") for lo, hi in slices]
    _KEEP.extend(parts)
    segs = (_ffi.BnpSeg * 2)(*[
        _ffi.BnpSeg(raw.data_ptr(), mean.data_ptr() + 4 * lo, invstd.data_ptr() + 4 * lo, beta.data_ptr() + 4 * lo,
                    part.data_ptr(), lo, hi, lo, cin, hi - lo, 0) for (lo, hi), part in zip(slices, parts)])
    wsb = L.jr_conv2d_workspace_size(ctypes.byref(d), 1, dt) + (1 << 20)
    ws = torch.zeros(wsb // 4 + 4, device="cuda")
    _KEEP.append(ws)
    _ffi.check("dgrad", L.jr_conv2d_bwd_data(ctypes.byref(d), dt, dy.data_ptr(), W.data_ptr(), dx_ref.data_ptr(),
                                             accumulate, ws.data_ptr(), wsb, None))
    _ffi.check("dgrad_bnp", L.jr_conv2d_bwd_data_bnp(ctypes.byref(d), dt, dy.data_ptr(), W.data_ptr(),
                                                     dx_bnp.data_ptr(), accumulate, 2, ctypes.byref(segs),
                                                     ws.data_ptr(), wsb, None))
    torch.cuda.synchronize()
    assert torch.equal(dx_ref, dx_bnp)
    # oracle terms on the stored values, jr_bn.hip's fp32 rounding of xhat / the mask
    DX = _host(dx_ref).reshape(-1, cin)
    X = raw.float().cpu().numpy().reshape(-1, cin)
    mu, isd, be = (t.cpu().numpy() for t in (mean, invstd, beta))
    xh = ((X - mu).astype(np.float32) * isd).astype(np.float32)
    g = np.where((xh + be).astype(np.float32) > 0, DX, 0.0)
    s0, s1 = g.sum(0), (g * xh.astype(np.float64)).sum(0)
    a0, a1 = np.abs(g).sum(0), np.abs(g * xh).sum(0)
    for (lo, hi), part in zip(slices, parts):
        c = hi - lo
        pr = part.cpu().numpy().reshape(2, c, P)
        assert np.all(np.abs(pr[0].sum(1) - s0[lo:hi]) <= 2e-5 * a0[lo:hi] + 1e-30)
        assert np.all(np.abs(pr[1].sum(1) - s1[lo:hi]) <= 2e-5 * a1[lo:hi] + 1e-30)
        # finalize + apply from the partials == the three-launch backward
        m = n * h * w
        dbeta_a = torch.zeros(c, device="cuda")
        dbeta_b = torch.zeros(c, device="cuda")
        out_a = torch.zeros(m * c, dtype=tdt, device="cuda")
        out_b = torch.zeros(m * c, dtype=tdt, device="cuda")
        _KEEP.extend([dbeta_a, dbeta_b, out_a, out_b])
        bws = max(L.jr_bn_workspace_size(m, c), 8 * c)
        bw = torch.zeros(bws // 4 + 4, device="cuda")
        _KEEP.append(bw)
        seg = _ffi.BnSeg(dx_ref.data_ptr(), lo, cin, c, beta.data_ptr() + 4 * lo, dbeta_a.data_ptr())
        # x / dx: the slice of raw; dx written with the same slice geometry -> out buffers of stride cin
        outa = torch.zeros(m * cin, dtype=tdt, device="cuda")
        outb = torch.zeros(m * cin, dtype=tdt, device="cuda")
        _KEEP.extend([outa, outb])
        _ffi.check("bwd_parts", L.jr_bn_relu_bwd_parts(bdt, 1, ctypes.byref(seg), part.data_ptr(), P, raw.data_ptr(),
                                                       lo, cin, m, c, mean.data_ptr() + 4 * lo,
                                                       invstd.data_ptr() + 4 * lo, outa.data_ptr(), bw.data_ptr(),
                                                       bws, None))
        seg.dbeta = dbeta_b.data_ptr()
        _ffi.check("bwd_multi", L.jr_bn_relu_bwd_multi(bdt, 1, ctypes.byref(seg), raw.data_ptr(), lo, cin, m, c,
                                                       mean.data_ptr() + 4 * lo, invstd.data_ptr() + 4 * lo,
                                                       outb.data_ptr(), bw.data_ptr(), bws, None))
        torch.cuda.synchronize()
        da, db = dbeta_a.cpu().numpy(), dbeta_b.cpu().numpy()
        assert np.all(np.abs(da - db) <= 2e-5 * a0[lo:hi] + 1e-30)
        ya = _host(outa).reshape(m, cin)[:, lo:hi]
        yb = _host(outb).reshape(m, cin)[:, lo:hi]
        tol = 1e-5 if f32 else 2.0 ** -7
        assert np.max(np.abs(ya - yb)) <= tol * np.max(np.abs(yb)), (np.max(np.abs(ya - yb)), np.max(np.abs(yb)))


def test_bnp_rejects_bad_slices():
    from jr import _ffi
    _ffi.init(0)
    L = _ffi.load()
    d = _ffi.ConvDesc(1, 8, 8, 64, 32, 3, 3, 1, 1, 1, 1, 8, 8, 0, 64, 0, 32)
    buf = torch.zeros(1 << 16, device="cuda")
    _KEEP.append(buf)
    p = buf.data_ptr()
    bad = [
        _ffi.BnpSeg(p, p, p, p, p, 0, 72, 0, 64, 72, 0),     # past c_in
        _ffi.BnpSeg(p, p, p, p, p, 16, 16, 0, 64, 16, 0),    # empty
        _ffi.BnpSeg(p, p, p, p, p, 0, 32, 40, 64, 32, 0),    # raw slice past its stride
        _ffi.BnpSeg(p, p, p, p, p, 0, 32, 0, 64, 16, 0),     # past the launch set
        _ffi.BnpSeg(p, p, p, p, p, 16, 64, 16, 64, 48, 0),   # not on a 32-channel boundary
    ]
    for sg in bad:
        arr = (_ffi.BnpSeg * 1)(sg)
        assert L.jr_conv2d_bwd_data_bnp(ctypes.byref(d), 0, p, p, p, 0, 1, ctypes.byref(arr), p, 1 << 18, None) != 0
    two = (_ffi.BnpSeg * 2)(_ffi.BnpSeg(p, p, p, p, p, 0, 32, 0, 64, 32, 0),
                            _ffi.BnpSeg(p, p, p, p, p, 0, 64, 0, 64, 64, 0))
    assert L.jr_conv2d_bwd_data_bnp(ctypes.byref(d), 0, p, p, p, 0, 2, ctypes.byref(two), p, 1 << 18, None) != 0
    torch.cuda.synchronize()
