"""The block-output BN backwards in one launch set (jr_bn_relu_bwd_batch,
VERDICT r04 item 5): every layer of a batch is bitwise its own
jr_bn_relu_bwd_multi call (dx and dbeta; fp32 and bf16; single- and
multi-segment layers of the 35^2 / 17^2 / 8^2 shapes), the engine's training
steps with the batching on and off are bitwise equal, and the batched launch
refuses a layer past 512 reduce chunks."""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _lib():
    from jr import _ffi
    _ffi.init(0)
    return _ffi


LAYERS = [(64 * 17 * 17, (192,)), (64 * 17 * 17, (160,)), (64 * 8 * 8, (384,)), (64 * 35 * 35, (64,)),
          (64 * 8 * 8, (256, 128))]


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_batch_equals_per_layer(dt):
    ffi = _lib()
    L = ffi.load()
    code = ffi.JR_F32 if dt == "f32" else ffi.JR_BF16
    et = torch.float32 if dt == "f32" else torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(21)
    data = []
    for m, segs in LAYERS:
        c = sum(segs)
        x = torch.randn(m * c, device="cuda", generator=g).to(et)
        mean = torch.randn(c, device="cuda", generator=g) * 0.1
        inv = torch.rand(c, device="cuda", generator=g) + 0.5
        beta = torch.randn(c, device="cuda", generator=g) * 0.2
        dys = [torch.randn(m * s, device="cuda", generator=g).to(et) for s in segs]
        data.append((m, segs, c, x, mean, inv, beta, dys))
    out = {}
    for batched in (False, True):
        res = []
        layers = (ffi.BnBwdLayer * len(data))()
        keep = []
        for k, (m, segs, c, x, mean, inv, beta, dys) in enumerate(data):
            dbeta = torch.zeros(c, device="cuda")
            dx = torch.zeros(m * c, device="cuda", dtype=et)
            arr = (ffi.BnSeg * len(segs))()
            o = 0
            for j, (s, dy) in enumerate(zip(segs, dys)):
                arr[j] = ffi.BnSeg(dy.data_ptr(), 0, s, s, beta.data_ptr() + 4 * o, dbeta.data_ptr() + 4 * o)
                o += s
            res.append((dx, dbeta))
            keep.append(arr)
            if batched:
                layers[k].nseg = len(segs)
                for j in range(len(segs)):
                    layers[k].segs[j] = arr[j]
                layers[k].x, layers[k].x_c_off, layers[k].x_c_stride = x.data_ptr(), 0, c
                layers[k].m, layers[k].c = m, c
                layers[k].mean, layers[k].invstd, layers[k].dx = mean.data_ptr(), inv.data_ptr(), dx.data_ptr()
            else:
                wsb = L.jr_bn_workspace_size(m, c)
                ws = torch.zeros(wsb // 4 + 64, device="cuda")
                keep.append(ws)
                ffi.check("multi", L.jr_bn_relu_bwd_multi(code, len(segs), ctypes.byref(arr), x.data_ptr(), 0, c, m, c,
                                                          mean.data_ptr(), inv.data_ptr(), dx.data_ptr(),
                                                          ws.data_ptr(), wsb, None))
        if batched:
            wsb = L.jr_bn_relu_bwd_batch_workspace_size(len(data), ctypes.byref(layers))
            assert wsb > 0
            ws = torch.zeros(wsb // 4 + 64, device="cuda")
            ffi.check("batch", L.jr_bn_relu_bwd_batch(code, len(data), ctypes.byref(layers), ws.data_ptr(), wsb, None))
        torch.cuda.synchronize()
        out[batched] = [(dx.float().cpu().numpy(), db.cpu().numpy()) for dx, db in res]
    for (a, b), (c_, d) in zip(out[False], out[True]):
        assert np.array_equal(a, c_) and np.array_equal(b, d)
        assert np.abs(a).max() > 0 and np.isfinite(a).all()


def test_batch_refuses_large_layers():
    ffi = _lib()
    L = ffi.load()
    m, c = 64 * 147 * 147, 64                       # a stem shape: > 512 reduce chunks
    layers = (ffi.BnBwdLayer * 2)()
    x = torch.zeros(m * c, device="cuda")
    dy = torch.zeros(m * c, device="cuda")
    st = torch.zeros(4 * c, device="cuda")
    for k in range(2):
        layers[k].nseg = 1
        layers[k].segs[0] = ffi.BnSeg(dy.data_ptr(), 0, c, c, st.data_ptr(), st.data_ptr() + 4 * c)
        layers[k].x, layers[k].x_c_off, layers[k].x_c_stride, layers[k].m, layers[k].c = x.data_ptr(), 0, c, m, c
        layers[k].mean, layers[k].invstd, layers[k].dx = st.data_ptr(), st.data_ptr(), x.data_ptr()
    wsb = L.jr_bn_relu_bwd_batch_workspace_size(2, ctypes.byref(layers))
    ws = torch.zeros(wsb // 4 + 64, device="cuda")
    assert L.jr_bn_relu_bwd_batch(ffi.JR_F32, 2, ctypes.byref(layers), ws.data_ptr(), wsb, None) == ffi.JR_ERR_UNSUPPORTED


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_engine_bn_batch_is_bitwise(dtype, monkeypatch):
    from jr import synth
    from jr.engine import Engine
    x, y = synth.fundus_batch(5, 6, 107), synth.labels(5, 6)
    out = {}
    for on in ("0", "1"):
        monkeypatch.setenv("JR_BN_BATCH", on)
        e = Engine(6, 107, 107, dtype=dtype, seed=4)
        _, bwd, _, _, _ = e._build_calls(6)
        nb = sum(1 for c in bwd if c.fn == e.lib.jr_bn_relu_bwd_batch)
        assert (nb >= 10) == (on == "1"), nb          # one per Inception block
        e.set_batch(x, y)
        losses = []
        for _ in range(3):
            e.train_step()
            losses.append(e.loss_value())
        out[on] = (losses, e.params_numpy())
    assert out["0"][0] == out["1"][0]
    assert np.array_equal(out["0"][1], out["1"][1])
