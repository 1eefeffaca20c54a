"""jr.plan on CPU: sibling-conv fusion groups, the internal parameter layout
and its Keras-layout round trip, and the ordering invariant the bucketed
all-reduce relies on (jr.dist: when a conv launch's backward is done, every
parameter at offsets >= its kernel offset is final)."""
import numpy as np
import pytest

from jr.inception import build_inception_v3
from jr.init import init_params, param_layout
from jr.plan import build_plan, sibling_groups


@pytest.fixture(scope="module")
def g():
    return build_inception_v3()


def test_sibling_groups_are_the_inception_branch_heads(g):
    groups = sibling_groups(g)
    # mixed0-2 (3 each), mixed4-7 (3 each), mixed8 (2), mixed9-10 (3 each)
    assert [len(m) for m in groups] == [3] * 3 + [3] * 4 + [2] + [3] * 2
    assert [sum(n.cout for n in m) for m in groups] == [176] * 3 + [448, 512, 512, 576] + [384] + [1152] * 2
    for m in groups:
        assert len({n.x for n in m}) == 1 and all(n.kh == n.kw == n.stride == 1 for n in m)
    plan = build_plan(g)
    assert len(plan.units) == 94 - sum(len(m) - 1 for m in groups)
    assert sum(len(u.members) for u in plan.units) == 94


@pytest.mark.parametrize("fuse", [True, False])
def test_layout_round_trip(g, fuse):
    plan = build_plan(g, fuse)
    flat = init_params(g, 3)
    flat += np.arange(flat.size, dtype=np.float32) * 1e-6   # distinct values everywhere
    _, total = param_layout(g.params)
    padding = np.ones(total, bool)
    for name, shape, off, size in param_layout(g.params)[0]:
        padding[off:off + size] = False
    flat[padding] = 0
    internal = plan.to_internal(g, flat)
    assert internal.size == plan.nparam
    assert np.array_equal(plan.to_keras(g, internal), flat)
    if not fuse:
        assert np.array_equal(internal, flat)           # identical to the Keras layout


def test_fused_kernel_block_is_the_concatenation(g):
    plan = build_plan(g)
    flat = init_params(g, 5)
    internal = plan.to_internal(g, flat)
    keras = {name: (off, size, shape) for name, shape, off, size in param_layout(g.params)[0]}
    for u in plan.units:
        if not u.fused:
            continue
        block = internal[u.koff:u.koff + u.cin * u.cout].reshape(u.cin, u.cout)
        cat = np.concatenate([flat[keras[f"{m.name}/kernel"][0]:][:keras[f"{m.name}/kernel"][1]]
                              .reshape(u.cin, m.cout) for m in u.members], axis=1)
        assert np.array_equal(block, cat)


@pytest.mark.parametrize("fuse", [True, False])
def test_reverse_walk_finalizes_suffixes(g, fuse):
    """Backward visits launches in reverse order of their first member; after
    launch u the set of final parameters must be exactly a suffix of the flat
    buffer starting at u's kernel offset (plus the dense head, done first)."""
    plan = build_plan(g, fuse)
    owner = {}   # internal offset -> launch that produces the gradient
    for name, shape, off, size in plan.layout:
        owner[off] = name
    final = set()
    dense = {plan.poff["dense/kernel"], plan.poff["dense/bias"]}
    final |= dense
    beta_off = {m.idx: plan.poff[f"batch_normalization_{m.idx + 1}/beta"] for u in plan.units for m in u.members}
    for u in reversed(plan.units):
        final.add(u.koff)
        final |= {beta_off[m.idx] for m in u.members}
        suffix = {off for _, _, off, _ in plan.layout if off >= u.koff}
        assert suffix <= final, (u.name, sorted(suffix - final)[:3])
    assert final == {off for _, _, off, _ in plan.layout}
