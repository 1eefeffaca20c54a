"""Data parallelism on the real engine: two ranks (torch.distributed gloo,
both on cuda:0 -- RCCL refuses two ranks on one device, the one-GPU box has
one) run Engine.train_step with jr.dist.BucketAllReduce, i.e. the engine's
own param_ready hooks over the fused internal parameter layout, buckets
issued during backward.  Reference: ONE process that computes both shards'
gradients with the same engine configuration, sums them (fp32 a + b, the
two-rank all-reduce) and applies the update with grad_scale 1/2.  After 3
steps the weights of both ranks equal the reference BITWISE.
"""
import os
import socket
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

B, RES, STEPS, WORLD = 4, 107, 3, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard(step, rank, b=B, res=RES):
    from jr import synth
    k = (step * WORLD + rank) * b
    return synth.fundus_batch(k, b, res), synth.labels(k, b, p=0.5)


def _rank(rank, port, outdir, dtype="f32", payload="f32", b=B, res=RES, steps=STEPS, math=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    from jr.dist import BucketAllReduce
    from jr.engine import Engine
    eng = Engine(b, res, res, seed=3, autotune=False, dtype=dtype, conv_math=math)
    ar = BucketAllReduce(eng, WORLD, bucket_bytes=8 << 20, payload=payload)
    losses, fences = [], []
    for step in range(steps):
        eng.set_batch(*_shard(step, rank, b, res))
        eng.train_step(allreduce=ar)
        losses.append(eng.loss_value())
        fences.append(ar.fences)
        if step == 0:   # the reduced (summed) gradient of step 0
            np.save(os.path.join(outdir, f"grad{rank}.npy"), eng.grads.cpu().numpy())
    np.save(os.path.join(outdir, f"params{rank}.npy"), eng.params.cpu().numpy())
    np.save(os.path.join(outdir, f"losses{rank}.npy"), np.array(losses))
    np.save(os.path.join(outdir, f"meta{rank}.npy"), np.array([len(ar.buckets), max(fences), eng.nlanes,
                                                               int(eng.tiles == "pinned")]))
    dist.barrier()
    dist.destroy_process_group()


# (dtype, payload, batch, resolution, steps): the 107^2 B=4 cases on the
# planner's tiles, and the bench workload itself -- 299^2 B=64, two lanes, the
# pinned MI355X tile tables (stream-K grids included) -- fp32 (x8) and bf16
CASES = [("f32", "f32", B, RES, STEPS, None), ("bf16", "f32", B, RES, STEPS, None),
         ("bf16", "bf16", B, RES, STEPS, None), ("f32", "f32", 64, 299, 2, None), ("bf16", "f32", 64, 299, 2, None),
         ("f32", "f32", 64, 299, 2, "x6h")]        # (the bench default: JR_F32_X6H convolutions)


@pytest.mark.parametrize("dtype,payload,b,res,steps,math", CASES)
def test_two_ranks_equal_one_process_averaging_shards(dtype, payload, b, res, steps, math):
    """fp32 and bf16 engines (configs 2 and 3), fp32 or bf16 gradient payload.
    The one-process reference sums the two shards' gradients exactly as the
    two-rank all-reduce does: fp32 a + b, or (bf16 payload) each shard's
    gradient rounded to bf16, added, the sum rounded to bf16 (gloo / RCCL sum
    bf16 values in fp32 -- exact for two terms -- and store bf16).  The
    buckets are issued from a stream that fences the lanes only at issue
    points with a ready bucket (at most one fence per bucket per step)."""
    import torch.multiprocessing as mp
    from jr.engine import Engine
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        ps = [ctx.Process(target=_rank, args=(r, port, d, dtype, payload, b, res, steps, math)) for r in range(WORLD)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(600)
        assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
        got = [np.load(os.path.join(d, f"params{r}.npy")) for r in range(WORLD)]
        got_losses = [np.load(os.path.join(d, f"losses{r}.npy")) for r in range(WORLD)]
        got_g0 = [np.load(os.path.join(d, f"grad{r}.npy")) for r in range(WORLD)]
        meta = [np.load(os.path.join(d, f"meta{r}.npy")) for r in range(WORLD)]
    for nb, fences, nl, pinned in meta:
        assert 1 <= fences <= nb and nl == 2
        assert pinned == int(res == 299)            # the bench workload runs its committed tile table
    ref = Engine(b, res, res, seed=3, autotune=False, dtype=dtype, conv_math=math)
    ref_losses = [[], []]
    for step in range(steps):
        gsum = None
        for r in range(WORLD):
            ref.set_batch(*_shard(step, r, b, res))
            ref.forward()
            ref.backward()
            ref.synchronize()
            ref_losses[r].append(ref.loss_value())
            g = ref.grads.clone()
            if payload == "bf16":
                g = g.to(torch.bfloat16).float()
            gsum = g if gsum is None else gsum + g
        if payload == "bf16":
            gsum = gsum.to(torch.bfloat16).float()
        ref.grads.copy_(gsum)
        torch.cuda.synchronize()          # copy_ ran on torch's stream, the update runs on the engine's
        if step == 0:
            want_g0 = gsum.cpu().numpy()
        ref.apply_update(grad_scale=1.0 / WORLD)
    ref.synchronize()
    want = ref.params.cpu().numpy()
    for r in range(WORLD):
        assert np.array_equal(got_losses[r], np.array(ref_losses[r])), (r, got_losses[r], ref_losses[r])
        bad = np.flatnonzero(got_g0[r] != want_g0)
        assert bad.size == 0, (r, bad.size, bad[:5], got_g0[r][bad[:5]], want_g0[bad[:5]])
    assert np.array_equal(got[0], got[1])                 # ranks stay bitwise identical
    assert np.array_equal(got[0], want)                   # == one process averaging the shards


@pytest.mark.parametrize("payload", ["f32", "bf16"])
def test_jr_comm_rccl_world1(payload, tmp_path):
    """libjr's own RCCL communicator (jr_comm_init_file / jr_allreduce_sum)
    at world 1 -- the one-GPU box cannot host two RCCL ranks: the sum over
    one rank is the identity for fp32 and bf16 buffers, and a training step
    whose buckets go through it (comm stream, bf16 or fp32 payload) equals
    the plain step (bf16 payload: the gradient rounded to bf16 once)."""
    from jr import _ffi
    from jr.dist import BucketAllReduce, JrComm
    from jr.engine import Engine
    comm = JrComm(0, 1, 0, uid_path=str(tmp_path / "uid"), run_id=f"test-{os.getpid()}")
    assert _ffi.load().jr_comm_world(comm.h) == 1
    x = torch.randn(1000, device="cuda")
    xb = x.to(torch.bfloat16)
    x0, xb0 = x.clone(), xb.clone()
    comm.allreduce(x.data_ptr(), x.numel(), _ffi.JR_F32, 0)
    comm.allreduce(xb.data_ptr(), xb.numel(), _ffi.JR_BF16, 0)
    torch.cuda.synchronize()
    assert torch.equal(x, x0) and torch.equal(xb, xb0)
    a = Engine(B, RES, RES, seed=3, autotune=False)
    b = Engine(B, RES, RES, seed=3, autotune=False)
    ar = BucketAllReduce(b, 1, bucket_bytes=8 << 20, comm=comm, payload=payload)
    for e in (a, b):
        e.set_batch(*_shard(0, 0))
    a.forward()
    a.backward()
    a.synchronize()
    if payload == "bf16":
        a.grads.copy_(a.grads.to(torch.bfloat16).float())
        torch.cuda.synchronize()
    a.apply_update()
    b.train_step(allreduce=ar)
    a.synchronize()
    b.synchronize()
    assert torch.equal(a.params, b.params)
    comm.close()


def _world1_rccl(outdir, dtype, math=None):
    """Child: a world-1 RCCL group (torch.distributed backend nccl) and the
    bench workload's DP step (bench.py --dp on) next to the plain step."""
    import socket as _s
    sk = _s.socket()
    sk.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(sk.getsockname()[1]), RANK="0", WORLD_SIZE="1")
    sk.close()
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    from jr.dist import BucketAllReduce
    from jr.engine import Engine
    a = Engine(64, 299, 299, seed=3, dtype=dtype, conv_math=math)
    b = Engine(64, 299, 299, seed=3, dtype=dtype, conv_math=math)
    ar = BucketAllReduce(b, 1)
    for step in range(2):
        for e in (a, b):
            e.set_batch(*_shard(step, 0, 64, 299))
        a.train_step()
        b.train_step(allreduce=ar)
    a.synchronize()
    b.synchronize()
    np.save(os.path.join(outdir, "w1.npy"), np.array([int(torch.equal(a.params, b.params)), len(ar.buckets),
                                                      ar.fences, int(a.tiles == "pinned")]))
    dist.destroy_process_group()


@pytest.mark.parametrize("dtype,math", [("f32", None), ("bf16", None), ("f32", "x6h")])
def test_world1_rccl_dp_step_equals_plain_step(dtype, math):
    """The DP machinery at the bench workload (299^2 B=64, two lanes, pinned
    tiles) over a real RCCL group of one rank: buckets issued from the feed
    stream during the backward, lane 0 waiting for them only before the
    optimizer -- bitwise the plain step, with at most one lane fence per
    bucket."""
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        p = mp.get_context("spawn").Process(target=_world1_rccl, args=(d, dtype, math))
        p.start()
        p.join(600)
        assert p.exitcode == 0, p.exitcode
        same, nb, fences, pinned = np.load(os.path.join(d, "w1.npy"))
    assert same == 1 and pinned == 1
    assert 1 <= fences <= nb
