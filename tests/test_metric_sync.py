"""Data-parallel metrics: ranks evaluate disjoint batches and sum their
streaming states (jr.session.Session.sync_metrics), so every rank reads the
single-pass Brier / AUC / confusion counts and takes the same early-stop
decision (train.py; CPU, gloo world 2)."""
import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp


class _Eng:
    units = 1


def _batches(seed, n=6, b=16):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        y = (rng.random((b, 1)) < 0.3).astype(np.float32)
        p = np.clip(0.6 * rng.random((b, 1)) + 0.3 * y, 0, 1).astype(np.float32)
        out.append((y, p))
    return out


def _run(sess, batches):
    sess.reset("tp", "fp", "fn", "tn", "brier", "auc")
    for y, p in batches:
        sess.update(y, p, "tp", "fp", "fn", "tn", "brier", "auc")
    sess.sync_metrics("tp", "fp", "fn", "tn", "brier", "auc")
    return sess.value("auc"), sess.value("brier"), sess.confusion_matrix()


def test_sync_equals_single_pass():
    from jr.session import Session
    batches = _batches(1)
    single = _run(Session(_Eng()), batches)
    a, b = Session(_Eng()), Session(_Eng())
    states = {}

    def fake_reduce(tag):
        def red(vec):
            states[tag] = vec
            return vec + states[1 - tag] if 1 - tag in states else vec
        return red
    # rank 1 first (its vec is stored), then rank 0 sums: then rank 1 again
    b.reduce = fake_reduce(1)
    _run(b, batches[1::2])
    a.reduce = fake_reduce(0)
    got = _run(a, batches[0::2])
    assert got[0] == single[0] and abs(got[1] - single[1]) < 1e-7
    np.testing.assert_array_equal(got[2], single[2])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from jr.session import Session
    sess = Session(_Eng())

    def red(vec):
        t = torch.from_numpy(vec)
        dist.all_reduce(t)
        return t.numpy()
    sess.reduce = red
    peak, waited, stopped_at = 0.0, 0, None
    for epoch in range(8):               # each rank sees different batches every epoch
        auc, _, _ = _run(sess, _batches(10 * epoch + rank))
        if auc < peak + 0.01:
            if waited == 2:
                stopped_at = epoch
                break
            waited += 1
        else:
            peak, waited = auc, 0
        dist.barrier()                   # a rank that stopped alone would hang here
    q.put((rank, stopped_at, peak))
    dist.destroy_process_group()


def test_ranks_agree_on_early_stop_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in ps])
    for p in ps:
        p.join(60)
    assert res[0][1:] == res[1][1:], res
