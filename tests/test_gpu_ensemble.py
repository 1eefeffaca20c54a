"""Grouped ensemble inference (BASELINE config 4: evaluate.py -lm over M
members).  jr_conv2d_fwd_bn_stats_grouped / jr_bn_relu_apply_grouped run M
members' layers in one launch each (member = blockIdx.y); jr.EnsembleEngine
strings them into the Inception-v3 forward.  Every member runs its own
per-member plan and batch statistics, so the results are BITWISE those of
the per-member path:
  * the grouped conv + statistics vs M single calls, f32 / x8 / bf16, with
    the planner's and forced split-K factors (the slab, partial and output
    member offsets), and the two-stage statistics combine (> 4,096 partials);
  * EnsembleEngine predictions vs one jr.Engine(train=False) per member, full
    and partial last batch, at 107^2 (planner tiles) and at the eval
    geometry 299^2 B=32 (the pinned eval tables).
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


def _lib():
    from jr import _ffi
    _ffi.init(0)
    return _ffi


def zeros(n, dtype=torch.float32):
    t = torch.zeros(int(n), dtype=dtype, device="cuda")
    _KEEP.append(t)
    return t


def _conv_case(ffi, L, dt, case, members, cfg=None, seed=3):
    n, h, w, cin, cout, kh, kw, s, pad = case
    ph, pw = ((kh - 1) // 2, (kw - 1) // 2) if pad == "same" else (0, 0)
    ho, wo = (h + 2 * ph - kh) // s + 1, (w + 2 * pw - kw) // s + 1
    q = 8 if dt == ffi.JR_BF16 else 4
    xs = (cin + q - 1) // q * q
    d = ffi.ConvDesc(n, h, w, cin, cout, kh, kw, s, s, ph, pw, ho, wo, 0, xs, 0, cout)
    at = torch.bfloat16 if dt == ffi.JR_BF16 else torch.float32
    g = torch.Generator(device="cuda").manual_seed(seed)
    xm = n * h * w * xs
    X = torch.randn(members * xm, device="cuda", generator=g).to(at)
    X.view(members, n * h * w, xs)[:, :, cin:] = 0
    if dt == ffi.JR_BF16:       # the bf16 filter operand: W^T [co][kh][kw][c8]
        c8 = (cin + 7) // 8 * 8
        wm = cout * kh * kw * c8
        Wt = (torch.randn(members, cout, kh, kw, c8, device="cuda", generator=g) * 0.1)
        Wt[..., cin:] = 0
        W = Wt.to(torch.bfloat16).reshape(-1)
    else:
        wm = kh * kw * cin * cout
        W = torch.randn(members * wm, device="cuda", generator=g) * 0.1
    ym = n * ho * wo * cout
    _KEEP.extend([X, W])
    if dt == ffi.JR_F32_X6H:    # magnitude words: member m's 64 at +64 m (jr.h grouped convention)
        words = zeros(64 * members)
        for m in range(members):
            words[64 * m + 3] = W[m * wm:(m + 1) * wm].abs().max()
        d.w_absmax = words.data_ptr()
        d.x_bound = float(X.abs().max())
    if cfg is not None:
        ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), 0, dt, 0, cfg))
    try:
        # (forced split-K factors may exceed the planner's workspace bound)
        extra = 0 if cfg is None else 4 * (cfg >> 8) * n * ho * wo * cout + (1 << 20)
        wsb = L.jr_conv2d_workspace_size_grouped(ctypes.byref(d), dt, members) + members * extra
        ws = zeros(wsb // 4 + 4)
        Yg, Sg = zeros(members * ym, at), zeros(members * 2 * cout)
        ffi.check("grouped", L.jr_conv2d_fwd_bn_stats_grouped(
            ctypes.byref(d), dt, members, X.data_ptr(), xm, W.data_ptr(), wm, Yg.data_ptr(), ym, 1e-3,
            Sg.data_ptr(), Sg.data_ptr() + 4 * cout, 2 * cout, ws.data_ptr(), wsb, None))
        ws1 = L.jr_conv2d_workspace_size(ctypes.byref(d), 0, dt) + extra
        w1 = zeros(ws1 // 4 + 4)
        esz = 2 if dt == ffi.JR_BF16 else 4
        for m in range(members):
            Y, S = zeros(ym, at), zeros(2 * cout)
            if dt == ffi.JR_F32_X6H:
                d.w_absmax = words.data_ptr() + 4 * 64 * m
            ffi.check("single", L.jr_conv2d_fwd_bn_stats(
                ctypes.byref(d), dt, X.data_ptr() + esz * m * xm, W.data_ptr() + esz * m * wm, Y.data_ptr(), 1e-3,
                S.data_ptr(), S.data_ptr() + 4 * cout, w1.data_ptr(), ws1, None))
            torch.cuda.synchronize()
            assert torch.equal(Yg[m * ym:(m + 1) * ym], Y), (case, cfg, m, "y")
            assert torch.equal(Sg[m * 2 * cout:(m + 1) * 2 * cout], S), (case, cfg, m, "stats")
            assert float(Y.float().abs().max()) > 0
    finally:
        if cfg is not None:
            ffi.check("reset", L.jr_conv2d_set_config(ctypes.byref(d), 0, dt, 0, -1))
        if dt == ffi.JR_F32_X6H:
            d.w_absmax = words.data_ptr()


CASES = [(4, 17, 17, 192, 192, 1, 7, 1, "same"), (4, 8, 8, 448, 384, 3, 3, 1, "same"),
         (4, 35, 35, 288, 64, 1, 1, 1, "same"), (3, 37, 37, 3, 32, 3, 3, 2, "valid")]


@pytest.mark.parametrize("dt", ["f32", "x8", "x6h", "bf16"])
@pytest.mark.parametrize("case", CASES)
def test_grouped_conv_equals_members(dt, case):
    ffi = _lib()
    L = ffi.load()
    code = {"f32": ffi.JR_F32, "x8": ffi.JR_F32_X8, "x6h": ffi.JR_F32_X6H, "bf16": ffi.JR_BF16}[dt]
    _conv_case(ffi, L, code, case, 3)
    for sp in (1, 4):                    # forced split-K: slab / partial member regions
        _conv_case(ffi, L, code, case, 3, cfg=0 | (sp << 8))


def test_grouped_conv_two_stage_statistics():
    """> 4,096 statistics partials (conv1 at B=16): the two-stage combine runs
    per member too."""
    ffi = _lib()
    L = ffi.load()
    # tiles of 256 rows in 4 waves: 64-row partials, 5,550 of them
    for code, tile in ((ffi.JR_F32_X8, 2), (ffi.JR_BF16, 4)):
        _conv_case(ffi, L, code, (16, 299, 299, 3, 32, 3, 3, 2, "valid"), 2, cfg=tile | (1 << 8))


@pytest.mark.parametrize("dtype,math", [("f32", None), ("bf16", None), ("f32", "x6h")])
@pytest.mark.parametrize("res,B,M", [(107, 8, 3), (299, 32, 2)])
def test_ensemble_engine_equals_engines(dtype, math, res, B, M):
    from jr import synth
    from jr.engine import Engine
    from jr.ensemble import EnsembleEngine
    from jr.inception import build_inception_v3
    from jr.init import init_params
    g = build_inception_v3(res, res)
    params = [init_params(g, 40 + m) for m in range(M)]
    ens = EnsembleEngine(params, B, res, res, dtype=dtype, conv_math=math)
    for n in (B, 5):                      # full and partial last batch
        x, y = synth.fundus_batch(100, n, res), synth.labels(100, n, p=0.3)
        ens.set_batch(x, y)
        ens.forward(n)
        got = ens.predictions(n)
        assert got.shape == (M, n, 1)
        for m in range(M):
            e = Engine(B, res, res, dtype=dtype, train=False, seed=0, conv_math=math)
            e.load_params(params[m])
            e.set_batch(x, y)
            e.forward(n)
            want = e.predictions(n)
            assert np.array_equal(got[m], want), (dtype, math, res, n, m, np.abs(got[m] - want).max())
            del e
        assert len({got[m].tobytes() for m in range(M)}) == M     # the members differ


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_ensemble_fused_bn_maxpool_is_bitwise(dtype):
    """The stem's BN + ReLU inside its max-pools for every member in one launch
    (jr_bn_relu_maxpool3x3s2_fwd_grouped): predictions bitwise those of the
    separate grouped apply + max-pool, full and partial batch."""
    from jr import synth
    from jr.ensemble import EnsembleEngine
    from jr.inception import build_inception_v3
    from jr.init import init_params
    g = build_inception_v3(107, 107)
    params = [init_params(g, 60 + m) for m in range(3)]
    e = {f: EnsembleEngine(params, 6, 107, 107, dtype=dtype, fuse_pool=f) for f in (True, False)}
    assert len(e[True].pool_fused) == 2 and not e[False].pool_fused
    for n in (6, 4):
        x = synth.fundus_batch(200, n, 107)
        out = {}
        for f, eng in e.items():
            eng.set_batch(x)
            eng.forward(n)
            out[f] = eng.predictions(n)
        assert np.array_equal(out[True], out[False]), (dtype, n)


def test_ensemble_ten_members_grouped_equals_engines():
    """BASELINE config 4's member count: ten members in
    one EnsembleEngine at 107^2, bitwise ten jr.Engine(train=False), full and
    partial batch."""
    from jr import synth
    from jr.engine import Engine
    from jr.ensemble import EnsembleEngine
    from jr.inception import build_inception_v3
    from jr.init import init_params
    res, B, M = 107, 8, 10
    g = build_inception_v3(res, res)
    params = [init_params(g, 300 + m) for m in range(M)]
    ens = EnsembleEngine(params, B, res, res, dtype="f32")
    e = Engine(B, res, res, dtype="f32", train=False, seed=0)
    for n in (B, 3):
        x = synth.fundus_batch(500 + n, n, res)
        ens.set_batch(x)
        ens.forward(n)
        got = ens.predictions(n)
        for m in range(M):
            e.load_params(params[m])
            e.set_batch(x)
            e.forward(n)
            assert np.array_equal(got[m], e.predictions(n)), (n, m)
        assert len({got[m].tobytes() for m in range(M)}) == M


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("res,B", [(107, 8), (299, 32)])
def test_ensemble_lanes_are_bitwise_one_lane(dtype, res, B):
    """EnsembleEngine on two branch lanes, each with its own conv workspace
    (split-K slabs, stream-K partials, statistics partials: the resource
    ("ws", lane)): every pass bitwise the one-lane predictions, full and
    partial batch (the round-4 prototype shared one workspace between the
    lanes, tools/ensemble_lanes_race.py)."""
    from jr import synth
    from jr.ensemble import EnsembleEngine
    from jr.inception import build_inception_v3
    from jr.init import init_params
    from jr.lanes import check_schedule
    g = build_inception_v3(res, res)
    params = [init_params(g, 80 + m) for m in range(3)]
    one = EnsembleEngine(params, B, res, res, dtype=dtype, lanes=1)
    two = EnsembleEngine(params, B, res, res, dtype=dtype, lanes=2)
    assert one.tiles == two.tiles
    for n in (B, 5):
        calls, _ = two._build_calls(n)
        check_schedule(calls)
        check_schedule(calls, precise=True)
        assert {c.lane for c in calls} == {0, 1}
        for k in range(3):
            x = synth.fundus_batch(700 + 40 * k, n, res)
            for e in (one, two):
                e.set_batch(x)
                e.forward(n)
            assert np.array_equal(one.predictions(n), two.predictions(n)), (dtype, res, n, k)
