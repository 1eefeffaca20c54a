"""conv2d_1 as a direct VALU convolution (csrc/jr_conv_direct.hip, VERDICT r04
item 4; opt-in, JR_CONV1_DIRECT=1, fp32 only -- see the kernel's notes): c_in
3 stored 4 fp32 wide, 3x3 stride 2 'valid', c_out 32, with the fused BN
statistics (one (mean, M2) partial per 1,024 output pixels).  Against the
fp64 oracle at the per-op bars of test_gpu_ops.py (fp32 outputs 5e-6 of
max|y|; mean 1e-5 of max|y|, invstd 1e-5 relative), on geometries whose last
block is partial; jr_conv2d_fwd (no statistics) writes the same y bitwise;
every member of a grouped launch is bitwise its own call.  The knob is read
once per process: test_direct_kernel_suite runs this module again in a child
process with JR_CONV1_DIRECT=1 (the checks skip in the parent).  (The direct
kernel replaces the GEMM for this geometry whatever tile id a table pins for
it; autotuning still times the GEMM configs.)"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import tf_ops as R

pytestmark = pytest.mark.gpu
DIRECT = os.environ.get("JR_CONV1_DIRECT") == "1"
inner = pytest.mark.skipif(not DIRECT, reason="run by test_direct_kernel_suite with JR_CONV1_DIRECT=1")
torch = pytest.importorskip("torch")
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


def _bf16(a):
    t = torch.as_tensor(np.asarray(a, np.float32)).to(torch.bfloat16)
    return t.to(torch.float32).numpy().astype(np.float64), t


@inner
@pytest.mark.parametrize("dt", ["x8", "f32"])
@pytest.mark.parametrize("n,h", [(2, 299), (3, 41), (1, 75)])
def test_conv1_direct_vs_fp64(dt, n, h):
    ffi = _lib()
    L = ffi.load()
    code = {"x8": ffi.JR_F32_X8, "f32": ffi.JR_F32, "bf16": ffi.JR_BF16}[dt]
    q = 8 if dt == "bf16" else 4
    rng = np.random.default_rng(n * 1000 + h)
    x = rng.uniform(0, 1, (n, h, h, 3))
    wt32 = (rng.standard_normal((3, 3, 3, 32)) / np.sqrt(27)).astype(np.float32)
    ho = (h - 3) // 2 + 1
    d = ffi.ConvDesc(n, h, h, 3, 32, 3, 3, 2, 2, 0, 0, ho, ho, 0, q, 0, 32)
    xp = np.zeros((n, h, h, q))
    if dt == "bf16":
        x, _ = _bf16(x)
        xp[..., :3] = x
        X = torch.as_tensor(xp.astype(np.float32)).to(torch.bfloat16).cuda()
        wq, _ = _bf16(wt32)
        W = torch.zeros(32 * 9 * 8, dtype=torch.bfloat16, device="cuda")     # the W^T copy [co][kh][kw][c8]
        Wm = torch.as_tensor(wt32).cuda()
        ffi.check("wprep", L.jr_conv_weights_bf16(Wm.data_ptr(), 3, 3, 3, 32, None, W.data_ptr(), None))
        _KEEP.append(Wm)
        ot = torch.bfloat16
    else:
        x = x.astype(np.float32).astype(np.float64)
        xp[..., :3] = x
        X = torch.as_tensor(xp.astype(np.float32)).cuda()
        wq = wt32.astype(np.float64)
        W = torch.as_tensor(wt32).cuda()
        ot = torch.float32
    _KEEP.extend([X, W])
    M = n * ho * ho
    wsb = L.jr_conv2d_workspace_size(ctypes.byref(d), 0, code)
    ws = torch.zeros(wsb // 4 + 64, device="cuda")
    Y = torch.zeros(M * 32, dtype=ot, device="cuda")
    Y2 = torch.zeros(M * 32, dtype=ot, device="cuda")
    st = torch.zeros(64, device="cuda")
    ffi.check("fwd+stats", L.jr_conv2d_fwd_bn_stats(ctypes.byref(d), code, X.data_ptr(), W.data_ptr(), Y.data_ptr(),
                                                    1e-3, st.data_ptr(), st.data_ptr() + 128, ws.data_ptr(), wsb,
                                                    None))
    ffi.check("fwd", L.jr_conv2d_fwd(ctypes.byref(d), code, X.data_ptr(), W.data_ptr(), Y2.data_ptr(), ws.data_ptr(),
                                     wsb, None))
    torch.cuda.synchronize()
    assert torch.equal(Y, Y2)
    ref = R.conv2d(x, wq, 2, "valid").reshape(M, 32)
    got = Y.float().cpu().numpy().astype(np.float64).reshape(M, 32)
    bar = 8e-3 if dt == "bf16" else 5e-6
    assert np.abs(got - ref).max() <= bar * np.abs(ref).max(), np.abs(got - ref).max() / np.abs(ref).max()
    s = st.cpu().numpy().astype(np.float64)
    # statistics of y as stored
    mean, var = got.mean(0), got.var(0)
    assert np.abs(s[:32] - mean).max() <= 1e-5 * np.abs(got).max()
    assert np.abs(s[32:] * np.sqrt(var + 1e-3) - 1).max() < 1e-5


@inner
@pytest.mark.parametrize("dt", ["x8"])
def test_conv1_direct_grouped_members_bitwise(dt):
    ffi = _lib()
    L = ffi.load()
    code = ffi.JR_F32_X8 if dt == "x8" else ffi.JR_BF16
    q, et = (4, torch.float32) if dt == "x8" else (8, torch.bfloat16)
    n, h, M_ = 2, 61, 3
    ho = (h - 3) // 2 + 1
    d = ffi.ConvDesc(n, h, h, 3, 32, 3, 3, 2, 2, 0, 0, ho, ho, 0, q, 0, 32)
    g = torch.Generator(device="cuda").manual_seed(3)
    xm, ym = n * h * h * q, n * ho * ho * 32
    wm = 3 * 3 * 3 * 32 if dt == "x8" else 32 * 9 * 8
    X = torch.rand(M_ * xm, device="cuda", generator=g).to(et)
    X.view(M_, n * h * h, q)[:, :, 3:] = 0
    W = (torch.randn(M_ * wm, device="cuda", generator=g) * 0.2).to(et)
    if dt == "bf16":
        W.view(M_, 32, 9, 8)[..., 3:] = 0
    wsb = L.jr_conv2d_workspace_size_grouped(ctypes.byref(d), code, M_)
    ws = torch.zeros(wsb // 4 + 64, device="cuda")
    Yg = torch.zeros(M_ * ym, dtype=et, device="cuda")
    Sg = torch.zeros(M_ * 64, device="cuda")
    ffi.check("grouped", L.jr_conv2d_fwd_bn_stats_grouped(
        ctypes.byref(d), code, M_, X.data_ptr(), xm, W.data_ptr(), wm, Yg.data_ptr(), ym, 1e-3, Sg.data_ptr(),
        Sg.data_ptr() + 128, 64, ws.data_ptr(), wsb, None))
    ws1 = L.jr_conv2d_workspace_size(ctypes.byref(d), 0, code)
    w1 = torch.zeros(ws1 // 4 + 64, device="cuda")
    esz = 4 if dt == "x8" else 2
    for m in range(M_):
        Y = torch.zeros(ym, dtype=et, device="cuda")
        S = torch.zeros(64, device="cuda")
        ffi.check("single", L.jr_conv2d_fwd_bn_stats(
            ctypes.byref(d), code, X.data_ptr() + esz * m * xm, W.data_ptr() + esz * m * wm, Y.data_ptr(), 1e-3,
            S.data_ptr(), S.data_ptr() + 128, w1.data_ptr(), ws1, None))
        torch.cuda.synchronize()
        assert torch.equal(Yg[m * ym:(m + 1) * ym], Y) and torch.equal(Sg[m * 64:(m + 1) * 64], S), m


@pytest.mark.skipif(DIRECT, reason="the child run itself")
def test_direct_kernel_suite():
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, "-m", "pytest", os.path.abspath(__file__), "-q", "-x", "-p", "no:cacheprovider",
                        "-m", "gpu"], cwd=os.path.dirname(here), capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, JR_CONV1_DIRECT="1"))
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "7 passed" in r.stdout and "failed" not in r.stdout, r.stdout[-2000:]
