"""The op-list Inception-v3 (jr.inception) matches the Keras topology the
reference instantiates (train.py:129-133; SURVEY.md App. A totals) and the
independently written oracle graph (oracle/inception_ref.py)."""
import numpy as np
import pytest


def test_totals_match_survey_appendix_a():
    from jr.inception import build_inception_v3
    g = build_inception_v3(299, 299)
    assert len(g.convs) == 94
    assert g.num_params() == 21_770_401
    assert g.macs_per_image() == 5_711_168_096
    assert g.bn_elems_per_image() == 8_967_488
    assert sum(n.cout for n in g.convs) == 17_216
    assert (g.bufs[g.output_buf].h, g.bufs[g.output_buf].c) == (8, 2048)
    g5 = build_inception_v3(587, 587)
    assert g5.macs_per_image() == 23_952_756_320
    assert g5.bufs[g5.output_buf].h == 17


def test_concat_slices_cover_each_block_exactly():
    from jr.inception import build_inception_v3
    g = build_inception_v3()
    cover = {}
    for n in g.nodes:
        cover.setdefault(n.y.buf, []).append((n.y.c_off, n.y.c_off + n.y.c))
    for bid, spans in cover.items():
        spans.sort()
        assert spans[0][0] == 0 and spans[-1][1] == g.bufs[bid].c, g.bufs[bid].name
        for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
            assert a1 == b0, g.bufs[bid].name


def test_param_layout_matches_oracle_graph_at_small_resolution():
    torch = pytest.importorskip("torch")
    from jr.inception import build_inception_v3
    from jr.init import init_params, unflatten
    from oracle.inception_ref import InceptionV3Ref
    g = build_inception_v3(75, 75)
    P = unflatten(g, init_params(g, 0))
    ref = InceptionV3Ref(P, torch.float64, requires_grad=False)   # asserts every kernel shape
    with torch.no_grad():
        logits, probs, _ = ref.forward(np.zeros((2, 75, 75, 3), np.float32) + 0.5)
    assert logits.shape == (2, 1) and ref._k == 94


def test_glorot_init_statistics():
    from jr.inception import build_inception_v3
    from jr.init import glorot_limit, init_params, unflatten
    g = build_inception_v3()
    P = unflatten(g, init_params(g, 3))
    w = P["conv2d_5/kernel"]
    lim = glorot_limit(w.shape)
    assert np.all(np.abs(w) <= lim) and abs(w.std() - lim / np.sqrt(3)) < 0.01 * lim
    assert np.all(P["batch_normalization_5/beta"] == 0) and np.all(P["dense/bias"] == 0)
    assert not np.array_equal(init_params(g, 0), init_params(g, 1))
    assert np.array_equal(init_params(g, 4), init_params(g, 4))
