"""JR_F32_X8W parity: the JR_F32_X8 kernels with the FILTER operand arriving
as its three exact bf16 HWIO planes (jr_conv_weights_x8p with no W^T),
activations and gradients fp32 and split in registers as in X8.

Same tile, same split-K factor => the same bf16 products in the same
per-accumulator order, so forward (plain and with the fused BN statistics)
and data gradient (every stride phase, overwrite and accumulate) are BITWISE
equal to JR_F32_X8 -- on every x8 tile config (the wave-uniform-tap kernels
and the generic ones: conv1's 3 channels, channel radices that are not a
multiple of BK), planner and forced split-K.  The fp32-MFMA tile ids need
the fp32 filter and fail loudly.  At the engine level a training step with
the planes equals the step without them, bit for bit.
"""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

X8, X8W = 2, 4
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


def dev(a):
    t = torch.as_tensor(np.ascontiguousarray(a)).to("cuda")
    _KEEP.append(t)
    return t


def zeros(n, dtype=torch.float32):
    t = torch.zeros(int(n), dtype=dtype, device="cuda")
    _KEEP.append(t)
    return t


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def hwio_planes(ffi, L, wt):
    kh, kw, cin, cout = wt.shape
    W = dev(wt)
    hw = zeros(3 * wt.size, torch.bfloat16)
    ffi.check("wprep x8w", L.jr_conv_weights_x8p(W.data_ptr(), kh, kw, cin, cout, hw.data_ptr(), None, None))
    return W, hw


def _desc(ffi, n, h, w, cin, cout, kh, kw, s, pad):
    ph, pw = ((kh - 1) // 2, (kw - 1) // 2) if pad == "same" else (0, 0)
    ho, wo = (h + 2 * ph - kh) // s + 1, (w + 2 * pw - kw) // s + 1
    xs = (cin + 3) // 4 * 4
    return ffi.ConvDesc(n, h, w, cin, cout, kh, kw, s, s, ph, pw, ho, wo, 0, xs, 0, cout), ho, wo, xs


def _set(ffi, L, d, s, cin, cfg):
    ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), 0, X8, 0, cfg))
    if cin % 4 == 0:
        for ph in range(s * s):
            ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), 1, X8, ph, cfg))


def _compare(ffi, L, case, cfg, seed=7):
    n, h, w, cin, cout, kh, kw, s, pad = case
    rng = np.random.default_rng(seed)
    d, ho, wo, xs = _desc(ffi, n, h, w, cin, cout, kh, kw, s, pad)
    x = np.zeros((n, h, w, xs), np.float32)
    x[..., :cin] = rng.standard_normal((n, h, w, cin))
    wt = (rng.standard_normal((kh, kw, cin, cout)) / np.sqrt(kh * kw * cin)).astype(np.float32)
    dy = rng.standard_normal((n, ho, wo, cout)).astype(np.float32)
    X, DY = dev(x), dev(dy)
    W, HW = hwio_planes(ffi, L, wt)
    if cfg is not None:
        _set(ffi, L, d, s, cin, cfg)
    wsb = max(L.jr_conv2d_workspace_size(ctypes.byref(d), op, X8) for op in range(2)) + (64 << 20)
    ws = zeros(wsb // 4 + 4)
    res = {}
    try:
        for dt, wp in ((X8, W), (X8W, HW)):
            Y, Y2 = zeros(n * ho * wo * cout), zeros(n * ho * wo * cout)
            st = zeros(2 * cout)
            ffi.check("fwd", L.jr_conv2d_fwd(ctypes.byref(d), dt, X.data_ptr(), wp.data_ptr(), Y.data_ptr(),
                                             ws.data_ptr(), wsb, None))
            ffi.check("fwd+stats", L.jr_conv2d_fwd_bn_stats(ctypes.byref(d), dt, X.data_ptr(), wp.data_ptr(),
                                                             Y2.data_ptr(), 1e-3, st.data_ptr(),
                                                             st.data_ptr() + 4 * cout, ws.data_ptr(), wsb, None))
            out = [host(Y), host(Y2), host(st)]
            if cin % 4 == 0:
                DX = zeros(x.size)
                ffi.check("dgrad", L.jr_conv2d_bwd_data(ctypes.byref(d), dt, DY.data_ptr(), wp.data_ptr(),
                                                        DX.data_ptr(), 0, ws.data_ptr(), wsb, None))
                out.append(host(DX))
                ffi.check("dgrad acc", L.jr_conv2d_bwd_data(ctypes.byref(d), dt, DY.data_ptr(), wp.data_ptr(),
                                                            DX.data_ptr(), 1, ws.data_ptr(), wsb, None))
                out.append(host(DX))
            res[dt] = out
    finally:
        if cfg is not None:
            _set(ffi, L, d, s, cin, -1)
    names = ("fwd", "fwd_bn_stats", "stats", "dgrad", "dgrad_acc")
    for name, a, b in zip(names, res[X8], res[X8W]):
        assert np.array_equal(a, b), (case, cfg, name, float(np.max(np.abs(a - b))))
    # and it is a convolution (the X8 kernels are checked against fp64 elsewhere)
    assert np.abs(res[X8][0]).max() > 0


CASES = [
    (2, 35, 35, 192, 64, 1, 1, 1, "same"),
    (2, 35, 35, 48, 64, 5, 5, 1, "same"),
    (2, 17, 17, 128, 192, 1, 7, 1, "same"),
    (2, 17, 17, 160, 160, 7, 1, 1, "same"),
    (2, 35, 35, 288, 384, 3, 3, 2, "valid"),
    (3, 17, 17, 192, 320, 3, 3, 2, "valid"),
    (2, 8, 8, 448, 384, 3, 3, 1, "same"),
    (2, 73, 73, 80, 192, 3, 3, 1, "valid"),
    (2, 37, 37, 3, 32, 3, 3, 2, "valid"),     # conv1: 3 channels, virtual padding (generic fwd)
    (1, 29, 31, 32, 48, 3, 3, 1, "same"),     # ragged M / N tails
]


@pytest.mark.parametrize("case", CASES)
def test_x8w_bitwise_x8_planner(case):
    ffi = _lib()
    _compare(ffi, ffi.load(), case, None)


@pytest.mark.parametrize("case", [(2, 17, 17, 64, 96, 3, 3, 1, "same"), (2, 17, 17, 48, 80, 3, 3, 2, "valid"),
                                  (2, 11, 11, 3, 32, 3, 3, 2, "valid"), (2, 8, 8, 128, 64, 1, 1, 1, "same"),
                                  (2, 19, 19, 80, 48, 1, 1, 1, "same")])
def test_x8w_bitwise_x8_every_tile(case):
    """Every x8 GEMM tile (ids 0..13; BK 16 and 32, so both the wave-uniform
    and the generic address paths of the filter planes), planner / forced
    split-K 1 and 3."""
    ffi = _lib()
    L = ffi.load()
    for t in range(14):
        for sp in (0, 1, 3):
            _compare(ffi, L, case, t | (sp << 8), seed=t)


def test_x8w_rejects_fp32_mfma_tiles():
    ffi = _lib()
    L = ffi.load()
    case = (2, 17, 17, 64, 96, 3, 3, 1, "same")
    n, h, w, cin, cout, kh, kw, s, pad = case
    d, ho, wo, xs = _desc(ffi, n, h, w, cin, cout, kh, kw, s, pad)
    W, HW = hwio_planes(ffi, L, np.ones((kh, kw, cin, cout), np.float32))
    X, Y = zeros(n * h * w * xs), zeros(n * ho * wo * cout)
    wsb = L.jr_conv2d_workspace_size(ctypes.byref(d), 0, X8)
    ws = zeros(wsb // 4 + 4)
    _set(ffi, L, d, s, cin, 14 + 3)
    try:
        rc = L.jr_conv2d_fwd(ctypes.byref(d), X8W, X.data_ptr(), HW.data_ptr(), Y.data_ptr(), ws.data_ptr(), wsb, None)
        assert rc == -3 and "X8W" in ffi.last_error()
        ffi.check("x8 fp32 tile", L.jr_conv2d_fwd(ctypes.byref(d), X8, X.data_ptr(), W.data_ptr(), Y.data_ptr(),
                                                  ws.data_ptr(), wsb, None))
    finally:
        _set(ffi, L, d, s, cin, -1)


@pytest.mark.parametrize("res,batch", [(107, 4), (299, 4)])
def test_engine_step_planes_equal_no_planes(res, batch):
    """Engine(conv_math='x8'): JR_X8W on (default) vs off -- logits, loss,
    every gradient and the updated parameters bitwise equal."""
    from jr import synth
    from jr.engine import Engine
    x, y = synth.fundus_batch(0, batch, res), synth.labels(0, batch, p=0.5)
    out = {}
    old = os.environ.get("JR_X8W")
    try:
        for flag in ("1", "0"):
            os.environ["JR_X8W"] = flag
            e = Engine(batch, res, res, seed=4, conv_math="x8")
            assert e.x8w == (flag == "1")
            e.set_batch(x, y)
            e.forward()
            e.backward()
            e.synchronize()
            g = e.grads.clone()
            e.apply_update()
            e.synchronize()
            out[flag] = (e.logits.cpu().numpy(), e.loss_value(), g.cpu().numpy(), e.params.cpu().numpy())
            del e
    finally:
        if old is None:
            os.environ.pop("JR_X8W", None)
        else:
            os.environ["JR_X8W"] = old
    for k, (a, b) in enumerate(zip(out["1"], out["0"])):
        assert np.array_equal(a, b), k
