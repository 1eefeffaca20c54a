"""BN + ReLU apply of a fused sibling launch's members in one launch
(jr_bn_relu_apply_multi): every member's output slice bitwise its own
jr_bn_relu_apply call (fp32, bf16; 17^2 / 35^2 / 8^2 shapes, members writing
into wider buffers at channel offsets), and the engine with the multi apply on
and off bitwise (three training steps and an eval forward)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _lib():
    from jr import _ffi
    _ffi.init(0)
    return _ffi


CASES = [(64 * 17 * 17, ((192, 768, 0), (160, 160, 0), (160, 320, 160))),
         (64 * 35 * 35, ((64, 256, 0), (48, 48, 0), (64, 64, 0))),
         (64 * 8 * 8, ((320, 1280, 0), (384, 384, 0), (256, 448, 192)))]   # (fp32: at most 1,024 channels)


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("case", CASES)
def test_apply_multi_equals_per_member(case, dt):
    ffi = _lib()
    L = ffi.load()
    code = ffi.JR_F32 if dt == "f32" else ffi.JR_BF16
    et = torch.float32 if dt == "f32" else torch.bfloat16
    m, members = case
    c = sum(mc for mc, _, _ in members)
    g = torch.Generator(device="cuda").manual_seed(c)
    x = torch.randn(m * c, device="cuda", generator=g).to(et)
    mean = torch.randn(c, device="cuda", generator=g) * 0.1
    inv = torch.rand(c, device="cuda", generator=g) + 0.5
    beta = torch.randn(c, device="cuda", generator=g) * 0.2
    outs = {}
    for multi in (False, True):
        ys = [torch.full((m * stride,), 7.0, device="cuda").to(et) for _, stride, _ in members]
        if multi:
            segs = (ffi.BnApplySeg * len(members))(*[
                ffi.BnApplySeg(y.data_ptr(), off, stride, mc, beta.data_ptr() + 4 * sum(q for q, _, _ in members[:i]))
                for i, ((mc, stride, off), y) in enumerate(zip(members, ys))])
            ffi.check("multi", L.jr_bn_relu_apply_multi(code, len(members), ctypes.byref(segs), x.data_ptr(), 0, c, m,
                                                        c, mean.data_ptr(), inv.data_ptr(), None))
        else:
            co = 0
            for (mc, stride, off), y in zip(members, ys):
                ffi.check("apply", L.jr_bn_relu_apply(code, x.data_ptr(), co, c, m, mc, mean.data_ptr() + 4 * co,
                                                      inv.data_ptr() + 4 * co, beta.data_ptr() + 4 * co, y.data_ptr(),
                                                      off, stride, None))
                co += mc
        torch.cuda.synchronize()
        outs[multi] = [y.float().cpu().numpy() for y in ys]
    for a, b in zip(outs[False], outs[True]):
        assert np.array_equal(a, b)
        assert (a != 7.0).any()


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_engine_apply_multi_is_bitwise(dtype, monkeypatch):
    from jr import synth
    from jr.engine import Engine
    x, y = synth.fundus_batch(7, 6, 107), synth.labels(7, 6)
    out = {}
    for on in ("0", "1"):
        monkeypatch.setenv("JR_APPLY_MULTI", on)
        e = Engine(6, 107, 107, dtype=dtype, seed=4)
        fwd, _, _, _, _ = e._build_calls(6)
        nm = sum(1 for c in fwd if c.fn == e.lib.jr_bn_relu_apply_multi)
        assert (nm >= 8) == (on == "1"), nm
        e.set_batch(x, y)
        losses = []
        for _ in range(3):
            e.train_step()
            losses.append(e.loss_value())
        ev = Engine(6, 107, 107, dtype=dtype, seed=0, train=False)
        ev.load_params(e.params_numpy())
        ev.set_batch(x)
        ev.forward()
        out[on] = (losses, e.params_numpy(), ev.predictions())
    assert out["0"][0] == out["1"][0]
    assert np.array_equal(out["0"][1], out["1"][1])
    assert np.array_equal(out["0"][2], out["1"][2])
