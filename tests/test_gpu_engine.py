"""Whole-network parity: jr.Engine (libjr kernels) vs the torch-CPU fp64
restatement oracle/inception_ref.py on identical seeded weights and synthetic
fundus inputs.  North-star tolerance: logits rel-err <= 1e-3."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _oracle_params(eng):
    from jr.init import unflatten
    return unflatten(eng.g, eng.params_numpy())


@pytest.mark.parametrize("res,batch", [(107, 3), (139, 2)])
def test_forward_and_one_step_match_oracle(res, batch):
    from jr.engine import Engine
    from jr import synth
    from oracle.inception_ref import InceptionV3Ref

    eng = Engine(batch, res, res, seed=1)
    imgs = synth.fundus_batch(0, batch, res)
    y = np.array([[1.0], [0.0], [1.0]][:batch], np.float32)
    eng.set_batch(imgs, y)
    P0 = _oracle_params(eng)
    ref = InceptionV3Ref(P0, torch.float64)
    x = imgs.astype(np.float32) * np.float32(1 / 255)
    state = {}
    loss_ref, probs_ref, grads_ref = ref.train_step(x, y, state)
    logits_ref = ref.last_logits

    eng.forward()
    eng.synchronize()
    logits = eng.logits[:batch].cpu().numpy().reshape(batch, 1)
    rel = np.max(np.abs(logits - logits_ref)) / max(np.max(np.abs(logits_ref)), 1e-3)
    assert rel <= 1e-3, (logits, logits_ref)
    assert abs(eng.loss_value() - loss_ref) <= 1e-3 * max(1.0, abs(loss_ref))

    eng.backward()
    eng.synchronize()
    from jr.init import unflatten
    G = unflatten(eng.g, eng.grads.cpu().numpy())
    worst = []
    for k, g_ref in grads_ref.items():
        g = G[k]
        scale = max(np.linalg.norm(g_ref), 1e-12)
        worst.append((np.linalg.norm(g - g_ref) / scale, k))
    worst.sort(reverse=True)
    assert worst[0][0] < 1e-2, worst[:5]

    eng.apply_update()
    P1 = unflatten(eng.g, eng.params_numpy())
    P1_ref = ref.params_numpy()
    for k in P1_ref:
        d = np.max(np.abs(P1[k] - P1_ref[k]))
        assert d < 1e-5, (k, d)


def test_graph_replay_equals_eager():
    """A captured HIP graph of the whole step gives bitwise the eager result."""
    from jr.engine import Engine
    from jr import synth
    imgs = synth.fundus_batch(0, 2, 107)
    y = np.array([[1.0], [0.0]], np.float32)
    a = Engine(2, 107, 107, seed=3)
    b = Engine(2, 107, 107, seed=3)
    for e in (a, b):
        e.set_batch(imgs, y)
    b.capture()
    for _ in range(3):
        a.train_step()
        b.replay()
    a.synchronize()
    b.synchronize()
    assert np.array_equal(a.params_numpy(), b.params_numpy())
    assert a.loss_value() == b.loss_value()


def test_partial_batch_uses_batch_statistics():
    """Eval of a partial last batch (evaluate.py batching) runs with B < plan."""
    from jr.engine import Engine
    from jr import synth
    from oracle.inception_ref import InceptionV3Ref
    eng = Engine(4, 107, 107, seed=2, train=False)
    imgs = synth.fundus_batch(10, 3, 107)
    eng.set_batch(imgs, np.zeros((3, 1), np.float32))
    eng.forward(3)
    p = eng.predictions(3)
    ref = InceptionV3Ref(_oracle_params(eng), torch.float64, requires_grad=False)
    with torch.no_grad():
        _, pr, _ = ref.forward(imgs.astype(np.float32) * np.float32(1 / 255))
    assert np.max(np.abs(p - pr.numpy())) < 1e-4
