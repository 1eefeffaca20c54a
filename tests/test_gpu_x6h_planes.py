"""JR_F32_X6H forward GEMMs reading pre-split filter planes
(jr_x6h_filter_planes + jr_conv_desc.w_planes, the Engine default) against
the same GEMMs splitting the filters in their K loop (JR_X6H_PLANES=0): the
planes hold the very terms SplitFrag16 forms, so three training steps at the
bench workload (299^2, B=64, pinned tables: split-K, stream-K and plain
grids, two lanes) and at a small one must be BITWISE equal -- loss,
parameters, momentum, predictions."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _run(size, batch, planes, monkeypatch):
    from jr import synth
    from jr.engine import Engine
    monkeypatch.setenv("JR_X6H_PLANES", "1" if planes else "0")
    e = Engine(batch, size, size, dtype="f32", seed=0, conv_math="x6h")
    assert (getattr(e, "wplanes", None) is not None) == planes
    if planes:
        assert e.planes_nseg > 50, e.planes_nseg      # every conv launch but conv2d_1 (c_in 3)
    x, y = synth.fundus_batch(0, batch, size), synth.labels(0, batch)
    e.set_batch(x, y)
    losses = []
    for _ in range(3):
        e.train_step()
        losses.append(e.loss_value())
    out = (losses, e.params_numpy(), e.accum.cpu().numpy(), e.predictions())
    del e
    torch.cuda.empty_cache()
    return out


@pytest.mark.parametrize("size,batch", [(107, 4), (299, 64)])
def test_filter_planes_bitwise_in_loop_split(size, batch, monkeypatch):
    l0, p0, a0, q0 = _run(size, batch, False, monkeypatch)
    l1, p1, a1, q1 = _run(size, batch, True, monkeypatch)
    assert np.isfinite(l0).all()
    assert l0 == l1, (l0, l1)
    assert np.array_equal(p0, p1) and np.array_equal(a0, a1) and np.array_equal(q0, q1)


def test_filter_planes_entry_rejects_bad_arguments():
    from jr import _ffi
    L = _ffi.load()
    assert L.jr_x6h_filter_planes(None, 1, None, None, None, None) != 0
    assert L.jr_x6h_filter_planes(None, 0, None, None, None, None) != 0
    assert os.environ.get("JR_X6H_PLANES", "1") in ("0", "1")
