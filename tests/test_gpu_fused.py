"""jr_conv2d_fwd_bn_stats: conv forward fused with the training-mode
BatchNormalization statistics of its output (Keras conv2d_bn, App. C Q1),
through the C-ABI, fp32 and bf16, with the statistics produced by the GEMM
epilogue (no split-K) and by the split-K reduce (forced split factors).

Checks: the raw output equals the oracle conv (fp32 1e-5 / bf16 8e-3 of
max |y|), and mean / invstd equal the fp64 statistics of the output AS
STORED (so the bf16 case is exact up to fp32 partial sums): mean within 1e-5
of max |y|, invstd within 1e-5 relative (biased variance, eps 1e-3).
"""
import ctypes

import numpy as np
import pytest

from oracle import tf_ops as R

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

_KEEP = []
WIDE0_BF16 = 25        # jr_conv_impl.h kCfgsBf16W: JR_BF16 ids after the 17 tiles and 8 halo configs


@pytest.fixture(autouse=True)
def _keep_alive():
    yield
    torch.cuda.synchronize()
    _KEEP.clear()


def _t(a, dtype):
    t = torch.as_tensor(np.ascontiguousarray(a, np.float32)).to(dtype).cuda()
    _KEEP.append(t)
    return t


CASES = [
    (2, 35, 35, 64, 96, 3, 3, 1, "same"),
    (3, 17, 17, 160, 192, 1, 7, 1, "same"),
    (2, 35, 35, 288, 384, 3, 3, 2, "valid"),
    (4, 8, 8, 448, 384, 3, 3, 1, "same"),
    (1, 29, 31, 32, 48, 3, 3, 1, "same"),    # ragged rows: partial groups with 0..WM rows
    (2, 37, 37, 3, 32, 3, 3, 2, "valid"),    # conv1 geometry (virtual channel padding)
]


@pytest.mark.parametrize("dtype", ["f32", "f32x8", "bf16"])
@pytest.mark.parametrize("case", CASES)
def test_conv_fwd_bn_stats(case, dtype):
    from jr import _ffi
    _ffi.init(0)
    L = _ffi.load()
    dt = {"f32": 0, "bf16": 1, "f32x8": 2}[dtype]
    f32 = dtype != "bf16"
    tdt = torch.float32 if f32 else torch.bfloat16
    q = 4 if f32 else 8
    n, h, w, cin, cout, kh, kw, s, pad = case
    rng = np.random.default_rng(sum(case[:8]))
    x = rng.standard_normal((n, h, w, cin)) + 0.5        # non-zero mean: exercises the centred M2
    wt = (rng.standard_normal((kh, kw, cin, cout)) / np.sqrt(kh * kw * cin)).astype(np.float32)
    cq = (cin + q - 1) // q * q
    xp = np.zeros((n, h, w, cq))
    xp[..., :cin] = x
    X = _t(xp, tdt)
    xr = X.double().cpu().numpy()[..., :cin]               # the input as the kernel sees it
    if f32:
        W = _t(wt, torch.float32)
        wr = wt.astype(np.float64)
    else:
        W32 = _t(wt, torch.float32)
        W = torch.zeros(cout * kh * kw * cq, dtype=torch.bfloat16, device="cuda")
        _KEEP.append(W)
        _ffi.check("wprep", L.jr_conv_weights_bf16(W32.data_ptr(), kh, kw, cin, cout, None, W.data_ptr(), None))
        wr = torch.as_tensor(wt).to(torch.bfloat16).double().numpy()
    ph, pw = ((kh - 1) // 2, (kw - 1) // 2) if pad == "same" else (0, 0)
    ho, wo = (h + 2 * ph - kh) // s + 1, (w + 2 * pw - kw) // s + 1
    d = _ffi.ConvDesc(n, h, w, cin, cout, kh, kw, s, s, ph, pw, ho, wo, 0, cq, 0, cout)
    ref = R.conv2d(xr, wr, s, pad)
    # + room for the forced split-K factors below (beyond the planner's own)
    wsb = L.jr_conv2d_workspace_size(ctypes.byref(d), 0, dt) + 5 * n * ho * wo * cout * 4 + (1 << 20)
    ws = torch.zeros(wsb // 4 + 4, device="cuda")
    _KEEP.append(ws)
    cfgs = [None, 0 | (1 << 8), 0 | (3 << 8), 3 | (1 << 8), 3 | (5 << 8)]
    if dtype == "bf16":     # the wide 8-wave tiles (ids after the halo configs): epilogue and split-K statistics
        wide0 = WIDE0_BF16
        cfgs += [wide0 | (1 << 8), (wide0 + 1) | (1 << 8), (wide0 + 6) | (1 << 8), (wide0 + 2) | (3 << 8)]
    for cfg in cfgs + [-1]:
        if cfg is not None:
            _ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), 0, dt, 0, cfg))
        Y = torch.zeros(n * ho * wo * cout, dtype=tdt, device="cuda")
        MEAN = torch.zeros(cout, device="cuda")
        INV = torch.zeros(cout, device="cuda")
        _KEEP.extend([Y, MEAN, INV])
        _ffi.check("fwd_bn_stats", L.jr_conv2d_fwd_bn_stats(ctypes.byref(d), dt, X.data_ptr(), W.data_ptr(),
                                                             Y.data_ptr(), 1e-3, MEAN.data_ptr(), INV.data_ptr(),
                                                             ws.data_ptr(), wsb, None))
        torch.cuda.synchronize()
        y = Y.double().cpu().numpy().reshape(ref.shape)
        scale = np.abs(ref).max()
        tol = 1e-5 if f32 else 8e-3
        assert np.abs(y - ref).max() <= tol * scale, (cfg, np.abs(y - ref).max() / scale)
        yf = y.reshape(-1, cout)
        mu = yf.mean(0)
        var = ((yf - mu) ** 2).mean(0)
        inv = 1.0 / np.sqrt(var + 1e-3)
        got_mu = MEAN.cpu().numpy().astype(np.float64)
        got_inv = INV.cpu().numpy().astype(np.float64)
        assert np.abs(got_mu - mu).max() <= 1e-5 * np.abs(yf).max(), (cfg, np.abs(got_mu - mu).max())
        assert np.abs(got_inv / inv - 1).max() <= 1e-5, (cfg, np.abs(got_inv / inv - 1).max())
