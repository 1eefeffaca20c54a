"""Data-parallel exchange logic on CPU: world_size 2 over gloo.

The GPU path runs the same BucketAllReduce over backend 'nccl' (RCCL); here
a stand-in replica exposes the engine's flat-gradient interface, and
backward's param_ready hooks are replayed in reverse layer order."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Replica:
    def __init__(self, layout, total, rank):
        self.layout, self.nparam = layout, total
        g = torch.Generator().manual_seed(100 + rank)
        self.grads = torch.randn(total, generator=g)
        self.stream = None


def test_buckets_cover_flat_gradient_in_reverse_order():
    from jr.dist import make_buckets
    from jr.inception import build_inception_v3
    from jr.init import param_layout
    layout, total = param_layout(build_inception_v3().params)
    b = make_buckets(layout, total, 24 << 20)
    assert b[0][1] == total and b[-1][0] == 0
    for (lo, hi), (lo2, hi2) in zip(b, b[1:]):
        assert hi2 == lo                                   # contiguous, descending
    starts = {off for _, _, off, _ in layout}
    assert all(lo in starts for lo, _ in b)                 # cut at tensor starts
    assert 3 <= len(b) <= 6                                 # ~87 MB / 24 MB
    assert 4 * (b[-1][1] - b[-1][0]) <= 2 << 20             # the unhidden last bucket kept small


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from jr.dist import BucketAllReduce
    from jr.inception import build_inception_v3
    from jr.init import param_layout
    g = build_inception_v3(107, 107)
    layout, total = param_layout(g.params)
    rep = _Replica(layout, total, rank)
    ar = BucketAllReduce(rep, world, bucket_bytes=4 << 20)
    ar.begin()
    issued = []
    convs = [off for name, _, off, _ in layout if name.startswith("conv2d_")]
    for off in reversed(convs):            # backward order: last conv first
        before = ar.next
        ar.param_ready(off)
        issued.append(ar.next - before)
    f_bwd = ar.fences
    scale = ar.finish()
    # the lanes are fenced once per issue point that has a ready bucket, never
    # at the other param_ready points (no per-conv join)
    assert f_bwd == sum(1 for x in issued if x)
    assert ar.fences - f_bwd in (0, 1) and ar.fences <= len(ar.buckets) < len(convs)
    q.put((rank, rep.grads.numpy() * scale, sum(1 for x in issued if x), len(ar.buckets)))
    dist.destroy_process_group()


def test_allreduce_world2_gloo_mean_and_overlap():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in ps], key=lambda t: t[0])
    for p in ps:
        p.join(60)
    from jr.inception import build_inception_v3
    from jr.init import param_layout
    _, total = param_layout(build_inception_v3(107, 107).params)
    want = (torch.randn(total, generator=torch.Generator().manual_seed(100)) +
            torch.randn(total, generator=torch.Generator().manual_seed(101))).numpy() / 2
    for rank, g, n_issue_points, n_buckets in res:
        np.testing.assert_allclose(g, want, rtol=1e-6, atol=1e-6)
        assert n_buckets >= 3 and n_issue_points >= 2      # buckets launched during backward
    np.testing.assert_array_equal(res[0][1], res[1][1])    # ranks bitwise identical


# ---------------------------------------------------------------- JrComm run id
def test_run_id_refuses_torchrun_default(monkeypatch):
    """torchrun without --rdzv-id exports TORCHELASTIC_RUN_ID='none' for every
    job: that must never tag an id file, nor MASTER_ADDR:PORT."""
    from jr.dist import resolve_run_id
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "none")
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", "29500")
    with pytest.raises(ValueError):
        resolve_run_id()
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "job42")
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "3")
    assert resolve_run_id() == "job42#3"
    assert resolve_run_id("explicit") == "explicit"


def _write_uid_file(path, run_id):
    import struct
    with open(path, "wb") as f:
        f.write(b"JRCOMMID" + struct.pack("<I", len(run_id)) + run_id.encode() + bytes(128))


def test_stale_none_tagged_id_file_is_not_joined(tmp_path, monkeypatch):
    """A stale id file tagged 'none' (an earlier default-torchrun job) at the
    path: under torchrun-like env vars JrComm refuses to guess a run id, and
    libjr's rank-1 poll with this job's run id ignores the stale file and
    times out instead of joining it (no GPU call is reached)."""
    from jr import _ffi
    from jr.dist import JrComm
    uid = str(tmp_path / "jr.uid")
    _write_uid_file(uid, "none")
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "none")
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", "29500")
    with pytest.raises(ValueError):
        JrComm(1, 2, 0, uid_path=uid, timeout_ms=200)
    with pytest.raises(_ffi.JRError, match="timed out"):
        JrComm(1, 2, 0, uid_path=uid, timeout_ms=300, run_id="nonce-abc")


def _nonce_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TORCHELASTIC_RUN_ID="none")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from jr.dist import resolve_run_id
    q.put((rank, resolve_run_id(), resolve_run_id()))
    dist.destroy_process_group()


def test_run_id_nonce_shared_over_group():
    """With a torch.distributed group every rank gets rank 0's fresh nonce
    (never 'none'); a second call draws a new one."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_nonce_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in ps])
    for p in ps:
        p.join(60)
    assert res[0][1] == res[1][1] and res[0][2] == res[1][2]
    assert res[0][1] != res[0][2] and res[0][1].startswith("nonce-") and "none" != res[0][1]
