"""The BN-statistics finalize folded into the BN apply:
jr_conv2d_fwd_bn_partials leaves the conv's single-stage (mean, M2)
partials in the workspace and jr_bn_relu_apply_stats combines each member
slice's channels (stats_combine8, the arithmetic k_stats_finalize8 uses)
before applying BN + ReLU.  Checked here:
  * per launch, against jr_conv2d_fwd_bn_stats + jr_bn_relu_apply on the
    same inputs: raw output, every member slice's activation, mean and
    invstd BITWISE equal -- planner tiles, a forced split-K factor (partials
    from the split-K reduce) and a stream-K grid (x8), fp32 (x8) and bf16;
  * the engine with the fold on and off: three training steps bitwise equal
    (loss, parameters) and the forward of an eval engine equal, f32 and bf16;
  * the layout query's geometry (P partials of R rows cover M)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _lib():
    from jr import _ffi
    _ffi.init(0)
    return _ffi


CASES = [  # n, h, w, cin, members' cout, kh, kw, stride, pad
    (8, 17, 17, 768, (192, 160, 160), 1, 1, 1, 0),
    (8, 17, 17, 160, (192,), 1, 7, 1, 3),
    (16, 8, 8, 448, (384,), 3, 3, 1, 1),
    (4, 35, 35, 288, (64, 48, 64), 1, 1, 1, 0),
]


@pytest.mark.parametrize("dt", ["x8", "bf16"])
@pytest.mark.parametrize("cfg", [None, "split", "sk"])
@pytest.mark.parametrize("case", CASES)
def test_fold_equals_separate_finalize(case, cfg, dt):
    ffi = _lib()
    L = ffi.load()
    n, h, w, cin, couts, kh, kw, s, pad = case
    cout = sum(couts)
    code = ffi.JR_F32_X8 if dt == "x8" else ffi.JR_BF16
    adt = ffi.JR_F32 if dt == "x8" else ffi.JR_BF16
    et = torch.float32 if dt == "x8" else torch.bfloat16
    ph, pw = (0, pad) if kh == 1 else (pad, 0) if kw == 1 else (pad, pad)
    ho, wo = (h + 2 * ph - kh) // s + 1, (w + 2 * pw - kw) // s + 1
    d = ffi.ConvDesc(n, h, w, cin, cout, kh, kw, s, s, ph, pw, ho, wo, 0, cin, 0, cout)
    if cfg == "sk" and dt == "bf16":
        pytest.skip("the bf16 stream-K ids are covered by test_gpu_streamk")
    force = {None: -1, "split": 0 | (4 << 8), "sk": 28 + 11}[cfg]
    if force >= 0:
        ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), 0, code, 0, force))
    try:
        g = torch.Generator(device="cuda").manual_seed(17)
        x = torch.randn(n * h * w * cin, device="cuda", generator=g).to(et)
        if dt == "bf16":
            wt = (torch.randn(cout * kh * kw * cin, device="cuda", generator=g) * 0.05).to(et)   # W^T operand
        else:
            wt = torch.randn(kh * kw * cin * cout, device="cuda", generator=g) * 0.05
        beta = torch.randn(cout, device="cuda", generator=g) * 0.1
        M = n * ho * wo
        wsb = L.jr_conv2d_workspace_size(ctypes.byref(d), 0, code)
        lay = ffi.BnPartials()
        ffi.check("layout", L.jr_conv2d_bn_partials_layout(ctypes.byref(d), code, ctypes.byref(lay)))
        assert lay.M == M and lay.N == cout and lay.P * lay.R >= M    # (a last row group may be empty)
        if cfg == "split":
            assert lay.P <= 512
        out = {}
        for fold in (False, True):
            ws = torch.zeros(wsb // 4 + 64, device="cuda")
            raw = torch.zeros(M * cout, device="cuda", dtype=et)
            st = torch.zeros(2 * cout, device="cuda")
            ys = [torch.zeros(M * c, device="cuda", dtype=et) for c in couts]
            if fold:
                ffi.check("partials", L.jr_conv2d_fwd_bn_partials(ctypes.byref(d), code, x.data_ptr(), wt.data_ptr(),
                                                                  raw.data_ptr(), ws.data_ptr(), wsb, None))
            else:
                ffi.check("stats", L.jr_conv2d_fwd_bn_stats(ctypes.byref(d), code, x.data_ptr(), wt.data_ptr(),
                                                            raw.data_ptr(), 1e-3, st.data_ptr(),
                                                            st.data_ptr() + 4 * cout, ws.data_ptr(), wsb, None))
            co = 0
            for c, y in zip(couts, ys):
                mp, ip = st.data_ptr() + 4 * co, st.data_ptr() + 4 * (cout + co)
                if fold:
                    ffi.check("apply_stats", L.jr_bn_relu_apply_stats(
                        adt, raw.data_ptr(), co, cout, M, c, ws.data_ptr() + lay.ws_offset, lay.P, lay.R, cout, co,
                        1e-3, mp, ip, beta.data_ptr() + 4 * co, y.data_ptr(), 0, c, None))
                else:
                    ffi.check("apply", L.jr_bn_relu_apply(adt, raw.data_ptr(), co, cout, M, c, mp, ip,
                                                          beta.data_ptr() + 4 * co, y.data_ptr(), 0, c, None))
                co += c
            torch.cuda.synchronize()
            out[fold] = (raw.clone(), st.clone(), [y.clone() for y in ys])
        (r0, s0, y0), (r1, s1, y1) = out[False], out[True]
        assert torch.equal(r0, r1)
        assert torch.equal(s0, s1), (s0 - s1).abs().max()
        for a, b in zip(y0, y1):
            assert torch.equal(a, b)
        m = r0.float().view(M, cout).double()
        assert torch.allclose(s0[:cout].double(), m.mean(0), rtol=0, atol=1e-4 * float(m.abs().max()))
    finally:
        if force >= 0:
            L.jr_conv2d_set_config(ctypes.byref(d), 0, code, 0, -1)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_engine_fold_is_bitwise(dtype):
    from jr import synth
    from jr.engine import Engine
    x, y = synth.fundus_batch(3, 6, 107), synth.labels(3, 6)
    out = {}
    for fold in (False, True):
        e = Engine(6, 107, 107, dtype=dtype, seed=4, fold_stats=fold)
        fwd, _, _, _, _ = e._build_calls(6)
        n_fold = sum(1 for c in fwd if c.name == "bn_relu" and c.fn == e.lib.jr_bn_relu_apply_stats)
        assert (n_fold > 0) == fold, n_fold
        e.set_batch(x, y)
        losses = []
        for _ in range(3):
            e.train_step()
            losses.append(e.loss_value())
        out[fold] = (losses, e.params_numpy())
        ev = Engine(6, 107, 107, dtype=dtype, seed=0, train=False, fold_stats=fold)
        ev.load_params(out[fold][1])
        ev.set_batch(x)
        ev.forward()
        out[fold] += (ev.predictions(),)
    assert out[False][0] == out[True][0]
    assert np.array_equal(out[False][1], out[True][1])
    assert np.array_equal(out[False][2], out[True][2])


_BWD_SCRIPT = r'''
import ctypes, sys
import numpy as np, torch
sys.path.insert(0, sys.argv[2])
from jr import _ffi
_ffi.init(0)
L = _ffi.load()
out = {}
for dt, m, segs in ((0, 18496, (192, 160, 160)), (1, 18496, (192, 160, 160)), (0, 4096, (384,)), (1, 4096, (384,)),
                    (0, 78400, (96,)), (1, 2000, (64, 32))):
    c = sum(segs)
    et = torch.float32 if dt == 0 else torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(m + c + dt)
    x = torch.randn(m * c, device="cuda", generator=g).to(et)
    mean = torch.randn(c, device="cuda", generator=g) * 0.1
    inv = torch.rand(c, device="cuda", generator=g) + 0.5
    beta = torch.randn(c, device="cuda", generator=g) * 0.2
    dys = [torch.randn(m * s, device="cuda", generator=g).to(et) for s in segs]
    dbeta = torch.zeros(c, device="cuda")
    dx = torch.zeros(m * c, device="cuda", dtype=et)
    arr = (_ffi.BnSeg * len(segs))()
    o = 0
    for k, (s, dy) in enumerate(zip(segs, dys)):
        arr[k] = _ffi.BnSeg(dy.data_ptr(), 0, s, s, beta.data_ptr() + 4 * o, dbeta.data_ptr() + 4 * o)
        o += s
    wsb = L.jr_bn_workspace_size(m, c)
    ws = torch.zeros(wsb // 4 + 64, device="cuda")
    _ffi.check("bwd", L.jr_bn_relu_bwd_multi(dt, len(segs), ctypes.byref(arr), x.data_ptr(), 0, c, m, c,
                                             mean.data_ptr(), inv.data_ptr(), dx.data_ptr(), ws.data_ptr(), wsb, None))
    torch.cuda.synchronize()
    out[f"dx_{dt}_{m}_{c}"] = dx.float().cpu().numpy()
    out[f"db_{dt}_{m}_{c}"] = dbeta.cpu().numpy()
np.savez(sys.argv[1], **out)
'''


def test_bn_backward_fold_is_bitwise(tmp_path):
    """The backward's finalize folded into its apply (k_bn_relu_bwd_apply_fold,
    JR_FOLD_BN_BWD) against the three launches (k_bn_finalize8 + apply):
    dx and dbeta bitwise, fp32 / bf16, fused-group segments, 17^2 / 8^2 /
    35^2 / partial shapes (the knob is read once per process: two
    processes)."""
    import os
    import subprocess
    import sys
    from conftest import PKG
    script = tmp_path / "bwd.py"
    script.write_text(_BWD_SCRIPT)
    res = {}
    for fold in ("0", "1"):
        f = tmp_path / f"out{fold}.npz"
        r = subprocess.run([sys.executable, str(script), str(f), PKG], capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, JR_FOLD_BN_BWD=fold))
        assert r.returncode == 0, r.stderr[-3000:]
        res[fold] = np.load(f)
    for k in res["0"].files:
        assert np.array_equal(res["0"][k], res["1"][k]), k
        assert np.isfinite(res["0"][k]).all() and np.abs(res["0"][k]).max() > 0, k
