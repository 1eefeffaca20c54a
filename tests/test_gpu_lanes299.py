"""Two lanes vs one lane of the full training step at the bench workload
(VERDICT r04 item 1c): Inception-v3 299^2, B=64, the PINNED tile tables
(stream-K x8 grids in fp32, split-K in bf16), the same seed and batch.
jr.lanes schedules every conflicting pair of calls across the two lanes, so
three steps on two lanes (the bench and train.py default) must leave
parameters, momentum, loss and predictions BITWISE those of one lane."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.mark.parametrize("dtype,math", [("f32", None), ("bf16", None), ("f32", "x6h")])
def test_two_lanes_bitwise_one_lane_299_b64_pinned(dtype, math):
    from jr import synth
    from jr.engine import Engine
    x, y = synth.fundus_batch(0, 64, 299), synth.labels(0, 64)
    out = {}
    for lanes in (1, 2):
        e = Engine(64, 299, 299, dtype=dtype, seed=0, lanes=lanes, conv_math=math)
        assert e.tiles == "pinned"
        if dtype == "f32":        # the fp32 table's stream-K grids are in play
            sk = sum(1 for f, wg, dg in e.conv_configs().values() for c in [f, wg, *dg]
                     if 28 <= (c & 255) < 42)
            assert sk > 50, sk
        e.set_batch(x, y)
        losses = []
        for _ in range(3):
            e.train_step()
            losses.append(e.loss_value())
        out[lanes] = (losses, e.params_numpy(), e.accum.cpu().numpy(), e.predictions())
        del e
        torch.cuda.empty_cache()
    (l1, p1, a1, q1), (l2, p2, a2, q2) = out[1], out[2]
    assert l1 == l2, (l1, l2)
    assert np.array_equal(p1, p2) and np.array_equal(a1, a2) and np.array_equal(q1, q2)
    assert np.isfinite(l1).all()


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
def test_config5_587_b64_two_lanes_bitwise_one_lane(dtype):
    """BASELINE config 5's per-GPU workload: 587^2, B=64,
    three steps.  bf16 runs its PINNED MI355X tile table (the split-K /
    stream-K grids the 587^2 bench line uses); fp32 (x8) has no committed
    587^2 table and runs the planner heuristic.  Two lanes are bitwise one
    lane, the loss is finite and the batch is being fitted."""
    from jr import synth
    from jr.engine import Engine
    x, y = synth.fundus_batch(0, 64, 587), synth.labels(0, 64)
    out = {}
    for lanes in (1, 2):
        e = Engine(64, 587, 587, dtype=dtype, seed=0, lanes=lanes)
        assert e.tiles == ("pinned" if dtype == "bf16" else "heuristic")
        e.set_batch(x, y)
        losses = []
        for _ in range(3):
            e.train_step()
            losses.append(e.loss_value())
        out[lanes] = (losses, e.params_numpy(), e.accum.cpu().numpy(), e.predictions())
        del e
        torch.cuda.empty_cache()
    (l1, p1, a1, q1), (l2, p2, a2, q2) = out[1], out[2]
    assert np.isfinite(l1).all() and l1[-1] < l1[0], l1
    assert l1 == l2, (l1, l2)
    assert np.array_equal(p1, p2) and np.array_equal(a1, a2) and np.array_equal(q1, q2)
