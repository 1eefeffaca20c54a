#!/usr/bin/env python3
"""bench.py — Inception-v3 299x299 training throughput on MI355X (libjr).

Metric (BASELINE.json): train images/sec, Inception-v3 299^2 bs64/GPU,
1-8 MI355X; % MFMA peak.  One step = forward + backward + gradient
all-reduce (N>1) + Nesterov update of one 64-image batch per GPU, the
reference's train.py:231-232 sess.run.  N=1 workload: BASELINE configs[1]
(fp32, batch 64, one GPU).  Synthetic fundus-shaped inputs (jr.synth),
resident in HBM before timing; Keras-default random init (App. C Q2).

  python bench.py [--gpus N --steps K --warmup W --dtype f32]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints ONE JSON line.  `roofline` is for the conv implicit-GEMM
family (the dominant kernels): algorithmic conv FLOPs per step / summed conv
op time per step, both from an instrumented pass (HIP events around every
conv call on the engine stream) run right after the timed region.
`cpu_baseline` times oracle/inception_ref.py (torch-CPU fp32 restatement,
kind "port") on the host cores for a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "jama16-retina-replication_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

# MI355X dense MFMA (MI355X_MICROARCH.md); x8 = eight bf16 MFMAs per fp32 product
PEAK_TFLOPS = {"f32": 157.3, "bf16": 2500.0, "x8": round(2500.0 / 8, 1), "x8p": round(2500.0 / 8, 1),
               "x6h": round(2500.0 / 6, 1)}
CONV_MATH = {"f32": "fp32 MFMA (v_mfma_f32_32x32x2_f32)",
             "x8": "fp32 via exact 3-way bf16 split, 8 bf16 MFMAs per product (all terms > 2^-32), "
                   "fp32 accumulate (JR_F32_X8)",
             "x8p": "fp32 via exact 3-way bf16 split done once per operand (jr_split_x8p planes), 8 bf16 MFMAs "
                    "per product, fp32 accumulate (JR_F32_X8P)",
             "x6h": "fp32 via a power-of-two-scaled 3-way fp16 split, 6 f16 MFMAs per product (dropped terms < "
                    "2^-32), fp32 accumulate (JR_F32_X6H)"}
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 200 timed steps (~5 s fp32, ~2 s bf16): long enough for the driver's
    # own GPU-busy sampler to see the timed window
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=None, help="per GPU (default 64 train, 32 eval)")
    ap.add_argument("--mode", default="train", choices=["train", "eval", "ensemble"],
                    help="eval: forward only with batch-statistics BN, the ensemble member pass of "
                         "evaluate.py:166-211 (BASELINE config 4); ensemble: evaluate.predict_all end to end "
                         "(TFRecord read + JPEG decode + every member's forward) over synthetic records")
    ap.add_argument("--members", type=int, default=10, help="ensemble mode: members resident on the GPU")
    ap.add_argument("--images", type=int, default=2048, help="ensemble mode: synthetic test images")
    ap.add_argument("--ens-lanes", type=int, default=2,
                    help="ensemble mode: branch lanes of the grouped EnsembleEngine (each with its own workspace)")
    ap.add_argument("--per-member", action="store_true",
                    help="ensemble mode: one engine per member instead of the grouped EnsembleEngine")
    ap.add_argument("--res", type=int, default=299)
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--conv-math", default="x6h", choices=["f32", "x8", "x8p", "x6h"],
                    help="dtype f32 only. x6h (default): fp32 tensors, products from a power-of-two-scaled 3-way "
                         "fp16 split, six f16 MFMAs (jr.h JR_F32_X6H; fp32-accurate, 4.5 %% faster than x8, "
                         "profiles/r06_ab_x6h_*.txt); x8: exact 3-way bf16 split, eight bf16 MFMAs (JR_F32_X8, "
                         "the library default); f32: fp32 MFMA")
    # eager launches on two lanes only: round 2 measured them 1.3-1.5 % faster
    # than HIP-graph replay (profiles/r02c_graph_ab.txt), and the measured path
    # keeps no graph code (Engine.capture stays an opt-in, separately tested API)
    ap.add_argument("--no-graph", action="store_true", help="no-op (eager is the only bench path; old commands)")
    ap.add_argument("--lanes", type=int, default=2, help="streams for branch-level concurrency (jr.lanes)")
    ap.add_argument("--tiles", default="pinned", choices=["pinned", "heuristic", "autotune"],
                    help="conv tiles: the committed MI355X table of this workload (train.py's default; "
                         "deterministic, bit-stable across boxes), the planner heuristic, or timed autotuning")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=64)
    ap.add_argument("--cpu-steps", type=int, default=2)
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--dp", default="auto", choices=["auto", "on", "off"],
                    help="bucketed gradient all-reduce in the step (jr.dist.BucketAllReduce): auto = only when "
                         "WORLD_SIZE > 1; on = also at N=1, over a world-1 RCCL group (the DP step timed on one GPU)")
    ap.add_argument("--dp-transport", default="jr", choices=["torch", "jr"],
                    help="libjr's own RCCL communicator (jr_comm_*, the default: measured +0.0 / +1.1 %% per fp32 / "
                         "bf16 step over the plain step at N=1, vs +1.1 / +3.7 %% through torch.distributed, "
                         "profiles/r06_dp_world1_ab.txt) or torch.distributed all_reduce (backend nccl = RCCL)")
    ap.add_argument("--no-defer-wgrad", action="store_true",
                    help="reduce each split-K filter gradient right after its GEMM (already the fp32 default; bf16 defers to one jr_wgrad_reduce)")
    return ap.parse_args()


def conv_roofline(eng, steps: int = 3):
    """Instrumented eager pass: HIP events (torch.cuda.Event on eng.stream)
    bracket every conv fwd/dgrad/wgrad call; returns (flops/step, conv s/step)."""
    from jr import _ffi
    fwd, bwd, opt, _, _ = eng._build_calls(eng.batch, 1)     # one lane: calls do not overlap
    # (wprep_bf16: the per-step filter prep the conv GEMMs read -- bf16 copies,
    # or x8's bf16 filter planes -- counted as conv time)
    conv_names = {"conv_fwd", "conv_dgrad", "conv_wgrad", "wgrad_reduce", "wprep_bf16"}
    flops = 0
    for n in eng.g.convs:
        m = n.macs_per_image() * eng.batch
        flops += 2 * m * ((2 if n.x == eng.g.input_buf else 3) if eng.train_mode else 1)
    pairs = []
    for _ in range(steps):
        for calls in (fwd, bwd, opt):
            for c in calls:
                if c.fn == "param_ready":
                    continue
                if c.name in conv_names:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(eng.stream)
                    rc = c.fn(*c.args)
                    e1.record(eng.stream)
                    pairs.append((e0, e1))
                else:
                    rc = c.fn(*c.args)
                if rc:
                    raise _ffi.JRError(c.name, rc, _ffi.last_error())
    eng.synchronize()
    t = sum(a.elapsed_time(b) for a, b in pairs) / 1e3 / steps
    return flops, t, len(pairs) // steps


FAMILY = {"bn_relu": "bn_relu_apply", "bn_relu_bwd": "bn_relu_bwd", "maxpool_fwd": "pool_fwd",
          "avgpool_fwd": "pool_fwd", "maxpool_bwd": "pool_bwd", "avgpool_bwd": "pool_bwd", "nesterov": "optimizer",
          "split_x8p": "split_x8p"}


def family_rates(eng, reps: int = 5) -> dict:
    """Achieved HBM rates of the bandwidth-bound kernel families over one
    step: every call of a family (BN+ReLU apply, BN+ReLU backward, pools
    fwd/bwd, the Nesterov update; x8p's operand splits) captured into ONE HIP
    graph on the engine stream and replayed back to back, timed with HIP
    events on that stream; algorithmic bytes = each call's declared reads +
    writes (jr.engine: e.g. BN apply 2 x M x C x elem, BN backward 3 passes,
    Nesterov 20 B/param).  Run after the timed region (the replays rewrite
    activations / scratch the next real step recomputes)."""
    from collections import defaultdict
    from jr import _ffi
    L = eng.lib
    fwd, bwd, opt, _, _ = eng._build_calls(eng.batch, 1)
    fam = defaultdict(list)
    for c in fwd + bwd + opt:
        if c.fn != "param_ready" and c.nbytes and c.name in FAMILY:
            fam[FAMILY[c.name]].append(c)
    out = {}
    for name, calls in fam.items():
        eng.synchronize()
        _ffi.check("jr_graph_begin", L.jr_graph_begin(eng._s))
        try:
            for c in calls:
                rc = c.fn(*c.args)
                if rc:
                    raise _ffi.JRError(c.name, rc, _ffi.last_error())
        finally:
            ex = __import__("ctypes").c_void_p()
            _ffi.check("jr_graph_end", L.jr_graph_end(eng._s, __import__("ctypes").byref(ex)))
        _ffi.check("jr_graph_launch", L.jr_graph_launch(ex, eng._s))     # warm-up
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(eng.stream)
        for _ in range(reps):
            _ffi.check("jr_graph_launch", L.jr_graph_launch(ex, eng._s))
        e1.record(eng.stream)
        eng.synchronize()
        L.jr_graph_destroy(ex)
        t = e0.elapsed_time(e1) / 1e3 / reps
        nbytes = sum(c.nbytes for c in calls)
        gbs = nbytes / t / 1e9
        out[name] = {"launches": len(calls), "ms_per_step": round(t * 1e3, 3), "bytes_per_step": nbytes,
                     "achieved_GBs": round(gbs, 1), "frac_of_8TBs": round(gbs / HBM_PEAK_GBS, 3)}
    return out


def pmc_traffic(dtype: str, B: int, res: int, math: str = "x8") -> dict:
    """HBM bytes of the conv family per training step from the committed
    rocprofv3 PMC summary of the same workload (tools/pmc_step.sh ->
    profiles/r01_pmc_<dtype>.json: FETCH_SIZE x 2 (gfx950 tallies 128-B
    requests at 64 B, MI355X_MICROARCH.md HBM section) + WRITE_SIZE, over the
    conv GEMM, split-K reduce and statistics kernels of one step; the fp32
    MFMA variant's summary is r01_pmc_f32mfma.json).  bench.py
    cannot run the profiler itself, so `traffic` is null without that file."""
    if (B, res) != (64, 299):
        return {}
    tag = {"f32": "f32mfma", "x8p": "f32x8p", "x6h": "f32x6h"}.get(math, "f32") if dtype == "f32" else dtype
    for rnd in ("r06", "r05", "r04", "r03", "r02c", "r02", "r01"):      # the newest committed summary of this workload
        p = os.path.join(ROOT, "profiles", f"{rnd}_pmc_{tag}.json")
        if os.path.exists(p):
            break
    else:
        return {}
    fam = json.load(open(p))["families"].get("conv", {})
    if "hbm_read_bytes" not in fam or "hbm_write_bytes" not in fam:
        return {}
    return {"traffic": round(fam["hbm_read_bytes"] + fam["hbm_write_bytes"]),
            "traffic_unit": "HBM bytes per step (conv family, PMC)", "traffic_source": os.path.relpath(p, ROOT)}


def cpu_share() -> int:
    """CPUs this process may actually use: its affinity mask, capped by a
    cgroup CPU quota (the GPU box gives each one-GPU job a 16-CPU share while
    os.cpu_count() and the affinity mask show the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")   # the box exports its share here too
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return n


def log(msg: str) -> None:
    """Progress on stderr (the JSON line alone goes to stdout)."""
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def cpu_baseline(args, res):
    from jr.inception import build_inception_v3
    from jr.init import init_params, unflatten
    from jr import synth
    from oracle.inception_ref import InceptionV3Ref
    # every core this process may run on (the job's CPU share; os.cpu_count()
    # is the whole machine's count, stated beside it)
    cores = cpu_share()
    torch.set_num_threads(cores)
    g = build_inception_v3(res, res)
    ref = InceptionV3Ref(unflatten(g, init_params(g, 0)), torch.float32)
    B = args.cpu_batch
    x = synth.fundus_batch(0, B, res).astype(np.float32) * np.float32(1 / 255)
    y = synth.labels(0, B)
    st = {}
    ref.train_step(x, y, st)   # warm-up
    t0 = time.perf_counter()
    for k in range(args.cpu_steps):
        ref.train_step(x, y, st)
        log(f"cpu baseline step {k + 1}/{args.cpu_steps} on {cores} threads")
    dt = time.perf_counter() - t0
    return {"value": round(B * args.cpu_steps / dt, 3), "unit": "images/sec", "cores": cores, "kind": "port",
            "host_cpu_count": os.cpu_count(),
            "sample": f"{args.cpu_steps} timed train steps (+1 warm-up) of batch {B} at {res}x{res} fp32, "
                      f"torch-CPU restatement oracle/inception_ref.py on {cores} threads = every CPU of this "
                      f"job's share (affinity mask capped by the cgroup quota; os.cpu_count() = {os.cpu_count()}) "
                      f"({dt:.1f} s)"}


def _write_records(out_dir: str, start: int, n: int, res: int, part: int) -> None:
    from jr import synth_records
    synth_records.write_split(out_dir, n, size=res, p=0.079, start=start, num_shards=1, name=f"test{part:02d}")


def dist_setup(args):
    """(rank, world, local, dist module or None): one process per GPU under
    torch.distributed.run; backend nccl = RCCL.  Rehearsal knobs for the N>1
    path on a one-GPU box (not for measurement): JR_BENCH_ONE_DEVICE=1 puts
    every rank on cuda:0, JR_DIST_BACKEND=gloo replaces RCCL (which refuses
    two ranks on one device)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0 and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    if os.environ.get("JR_BENCH_ONE_DEVICE") == "1":
        local = 0
    backend = os.environ.get("JR_DIST_BACKEND", "nccl")
    torch.cuda.set_device(local)
    dist = None
    if world > 1 or getattr(args, "dp", "auto") == "on":
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1 and "MASTER_PORT" not in os.environ:      # world-1 group, no launcher
            import socket
            sk = socket.socket()
            sk.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
            sk.close()
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local, dist


def gather_devices(dist, local: int) -> list:
    """The device index of every rank (n_gpus counts distinct devices: a
    rehearsal with every rank on cuda:0 is one GPU)."""
    if not dist or dist.get_world_size() == 1:
        return [local]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, local)
    return out


def max_over_ranks(dist, v: float) -> float:
    if not dist:
        return v
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([v], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def grouped_conv_roofline(ens, steps: int = 3):
    """The conv roofline of the grouped ensemble forward (BASELINE config 4):
    HIP events (on the stream each call is enqueued on) bracket every grouped
    conv + statistics launch, each run alone; algorithmic FLOPs = members x
    batch x 2 x MACs per image.  Every call of the pass, conv or not, runs
    with the device synchronised before and after it: the lanes' producer
    waits are not replayed here, so a fully serial pass is what keeps a BN
    apply or pool on one lane from racing its producer on the other (ADVICE
    r05), and a neighbour launch from sharing the CUs with a timed conv."""
    from jr import _ffi
    calls, _ = ens._build_calls(ens.batch)
    flops = sum(2 * n.macs_per_image() for n in ens.g.convs) * ens.batch * ens.members
    pairs = []
    for _ in range(steps):
        for c in calls:
            st = ens.lane_streams[c.lane]
            torch.cuda.synchronize()
            if c.name == "conv_fwd":
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                rc = c.fn(*c.args)
                e1.record(st)
                pairs.append((e0, e1))
            else:
                rc = c.fn(*c.args)
            torch.cuda.synchronize()
            if rc:
                raise _ffi.JRError(c.name, rc, _ffi.last_error())
    ens.synchronize()
    t = sum(a.elapsed_time(b) for a, b in pairs) / 1e3 / steps
    return flops, t, len(pairs) // steps


def ensemble_bench(args) -> dict:
    """BASELINE config 4: evaluate.predict_all (the -lm ensemble loop of
    evaluate.py: records read and decoded once per batch on the host, every
    resident member's forward on the GPU) timed end to end over synthetic
    fundus TFRecords, next to its two halves alone: the input pipeline
    (decode only) and the members' forwards on resident batches.  Under
    torch.distributed.run every rank takes the batches b = rank mod world in
    dataset order (evaluate.py's sharding, no data-path collective); the time
    is the max over ranks between two barriers, `value` = all images / it."""
    import multiprocessing as mp
    import shutil
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "jama16-retina-replication_amd"))
    import evaluate
    import lib.dataset
    from jr.engine import Engine
    rank, world, local, dist = dist_setup(args)
    B, res, n = args.batch or 32, args.res, args.images
    d = None
    try:
        if rank == 0:            # one copy of the test set for every rank of the node
            d = tempfile.mkdtemp(prefix="jr_ensemble_")
            parts = 8
            per = -(-n // parts)
            t0 = time.perf_counter()
            with mp.get_context("spawn").Pool(parts) as pool:
                pool.starmap(_write_records, [(d, k * per, min(per, n - k * per), res, k) for k in range(parts)
                                              if n - k * per > 0])
            log(f"{n} synthetic records in {time.perf_counter() - t0:.1f} s")
        if dist:
            box = [d]
            dist.broadcast_object_list(box, src=0)
            d = box[0]
        math = args.conv_math if args.dtype == "f32" else "bf16"
        if args.per_member:
            engines = [Engine(B, res, res, device=local, dtype=args.dtype, seed=m, train=False, conv_math=math,
                              tiles=args.tiles) for m in range(args.members)]
        else:                # every member's layer in one grouped launch (jr.ensemble)
            from jr.ensemble import EnsembleEngine
            from jr.inception import build_inception_v3
            from jr.init import init_params
            g = build_inception_v3(res, res)
            engines = EnsembleEngine([init_params(g, m) for m in range(args.members)], B, res, res, device=local,
                                     dtype=args.dtype, conv_math=math, tiles=args.tiles, lanes=args.ens_lanes)
        evaluate.predict_all(engines, d, B, rank, world)      # warm-up pass (decoder threads, tiles, caches)
        if dist:
            dist.barrier()
        t0 = time.perf_counter()
        preds, labels, ids = evaluate.predict_all(engines, d, B, rank, world)
        t_mine = time.perf_counter() - t0
        if dist:
            dist.barrier()
        t_all = max_over_ranks(dist, t_mine)
        n_mine = labels.shape[0]
        assert preds[0].shape[0] == n_mine and len(ids) == -(-n_mine // B)
        ds = lib.dataset.initialize_dataset(d, B, num_workers=evaluate.NUM_WORKERS, prefetch_buffer_size=2 * B,
                                            image_dim=[res, res], decode_dtype="uint8", shard=(rank, world))
        t0 = time.perf_counter()
        it = iter(ds)
        batches = [b for b in it]
        lib.dataset.close_iterator(it)
        t_dec = time.perf_counter() - t0
        x, y = batches[0]
        group = engines if args.per_member else [engines]
        for e in group:
            e.set_batch(x, y)
            e.forward()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(len(batches)):
            for e in group:
                e.forward()
        for e in group:
            e.synchronize()
        t_gpu = time.perf_counter() - t0
        roof = None
        if rank == 0 and not args.per_member and not args.no_roofline:
            flops, tconv, nconv = grouped_conv_roofline(engines)
            peak = PEAK_TFLOPS[math if math in ("x8", "x8p", "x6h") else args.dtype]
            ach = flops / tconv / 1e12
            roof = {"bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s",
                    "frac": round(ach / peak, 4), "traffic": None,
                    "kernel": f"grouped conv implicit-GEMM fwd + BN statistics, {args.members} members per launch "
                              f"({nconv} launches/forward)",
                    "conv_ms_per_forward": round(tconv * 1e3, 3),
                    "algorithmic_gflop_per_forward": round(flops / 1e9, 1)}
        devices = len({int(v) for v in gather_devices(dist, local)})
        rehearsal = world > 1 and (devices < world or dist.get_backend() != "nccl")
        if dist:
            dist.barrier()
    finally:
        if rank == 0 and d:
            shutil.rmtree(d, ignore_errors=True)
    M = args.members
    out = {
        "metric": f"ensemble eval images/sec, Inception-v3 {res}^2, {M} members, batch {B} (evaluate.py -lm)",
        "value": round(n / t_all, 2), "unit": "images/sec", "n_gpus": devices, "rehearsal": rehearsal,
        "steps": 1, "warmup": 1,
        "ms_per_step": round(t_all / -(-n // (B * world)) * 1e3, 3), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": args.dtype,
        "data": f"{n} synthetic fundus-shaped JPEG q=100 TFRecords at {res}x{res} (jr.synth_records), random Keras "
                f"init per member",
        "config": {"workload": f"evaluate.predict_all: {M} resident members x {-(-n // B)} batches of {B} over "
                               f"{world} rank(s) (batch b on rank b mod {world}), each batch read + decoded once "
                               f"(native JPEG, {evaluate.NUM_WORKERS} threads per rank) and run through every member "
                               f"({'one engine per member' if args.per_member else 'every member in one grouped launch per layer'})",
                   "model": "inception_v3", "global_batch": B * world, "seq_len": None,
                   "parallelism": f"dp{world} (batches sharded, no data-path collective)", "members": M,
                   "tiles": group[0].tiles, "grouped": not args.per_member,
                   "lanes": 1 if args.per_member else engines.nlanes},
        "member_images_per_s": round(n * M / t_all, 1),
        "decode_only_images_per_s": round(n_mine / t_dec, 1),
        "gpu_forward_only_images_per_s": round(n_mine / t_gpu, 1),
        "bound": "decode" if t_dec > t_gpu else "gpu",
        "roofline": roof,
    }
    if dist:
        dist.destroy_process_group()
    return out if rank == 0 else None


def _stdout_for_json_only() -> int:
    """Keep stdout for the ONE JSON line: everything else written to fd 1
    (RCCL prints its version banner to C stdout when a communicator comes
    up) goes to stderr; returns the fd the JSON line is written to."""
    sys.stdout.flush()
    fd = os.dup(1)
    os.dup2(2, 1)
    return fd


def emit(fd: int, out: dict) -> None:
    os.write(fd, (json.dumps(out) + "\n").encode())


def heartbeat(period: float = 50.0) -> None:
    """A progress line on stderr every `period` s from a daemon thread: long
    single passes (the 57,000-image ensemble in fp32 runs minutes between
    log lines) must not look hung to a watchdog."""
    import threading
    t0 = time.perf_counter()

    def run():
        while True:
            time.sleep(period)
            log(f"alive, {time.perf_counter() - t0:.0f} s")
    threading.Thread(target=run, daemon=True).start()


def main():
    args = parse()
    json_fd = _stdout_for_json_only()
    heartbeat()
    if args.mode == "ensemble":
        out = ensemble_bench(args)
        if out is not None:
            emit(json_fd, out)
        return
    rank, world, local, dist = dist_setup(args)

    from jr.engine import Engine
    from jr import synth
    from jr.dist import BucketAllReduce

    train = args.mode == "train"
    B, res = args.batch or (64 if train else 32), args.res
    math = args.conv_math if args.dtype == "f32" else "bf16"
    eng = Engine(B, res, res, device=local, dtype=args.dtype, seed=0, lanes=args.lanes, train=train,
                 conv_math=math, tiles=args.tiles, defer_wgrad=False if args.no_defer_wgrad else None)
    imgs = synth.fundus_batch(rank * B, B, res)
    labels = synth.labels(rank * B, B)
    eng.set_batch(imgs, labels)
    eng.synchronize()
    log(f"engine ready (rank {rank}/{world})")
    ar = comm = None
    transport = args.dp_transport
    if train and (world > 1 or args.dp == "on") and args.dp != "off":
        if transport == "jr":
            from jr import _ffi
            from jr.dist import JrComm
            try:
                comm = JrComm.from_torch_group(rank, world, local)
            except _ffi.JRError as e:      # (the same RCCL under torch.distributed then)
                log(f"libjr RCCL communicator unavailable ({e}); torch.distributed transport")
                transport = "torch"
        ar = BucketAllReduce(eng, world, comm=comm)
    use_graph = False

    def step():
        if train:
            eng.train_step(allreduce=ar)
        else:
            eng.forward()

    for i in range(args.warmup):
        step()
    eng.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    eng.synchronize()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = max_over_ranks(dist, time.perf_counter() - t0)
    loss = eng.loss_value() if train else float(np.mean(eng.predictions()))
    if not np.isfinite(loss):
        raise SystemExit(f"non-finite {'loss' if train else 'prediction'} {loss}")
    overlap = None
    if ar is not None:          # after the timed region: one traced step (timing events per issue point)
        ar.trace = True
        step()
        eng.synchronize()
        overlap = ar.overlap_ms()
        ar.trace = False

    devices = len({int(v) for v in gather_devices(dist, local)})
    rehearsal = world > 1 and (devices < world or dist.get_backend() != "nccl")
    out = None
    if rank == 0:
        imgs_s = B * world * args.steps / elapsed
        ms = elapsed / args.steps * 1e3
        log(f"timed {args.steps} steps: {ms:.3f} ms/step")
        roof = None
        if not args.no_roofline:
            flops, tconv, nconv = conv_roofline(eng)
            ach = flops / tconv / 1e12
            peak = PEAK_TFLOPS[math if math in ("x8", "x8p", "x6h") else args.dtype]
            roof = {"bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s",
                    "frac": round(ach / peak, 4), "traffic": None,
                    "kernel": f"conv implicit-GEMM {'fwd+dgrad+wgrad' if train else 'fwd'} ({nconv} calls/step)",
                    "conv_ms_per_step": round(tconv * 1e3, 3),
                    "algorithmic_gflop_per_step": round(flops / 1e9, 1)}
            if train:
                roof.update(pmc_traffic(args.dtype, B, res, math))
        hbm = None if args.no_roofline else family_rates(eng)
        out = {
            "metric": (f"train images/sec, Inception-v3 {res}^2 bs{B}/GPU" if train else
                       f"eval images/sec, Inception-v3 {res}^2 bs{B}/GPU (one ensemble member, batch-stat BN)"),
            "value": round(imgs_s, 2), "unit": "images/sec", "n_gpus": devices,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": args.dtype, "data": f"synthetic fundus-shaped uint8 {res}x{res}x3 (jr.synth), random Keras init",
            "config": {"workload": (f"Inception-v3 {res}x{res} {args.dtype} training, batch {B}/GPU, "
                                    f"Nesterov lr 3e-3 m 0.9" if train else
                                    f"Inception-v3 {res}x{res} {args.dtype} forward (evaluate.py), batch {B}/GPU, "
                                    f"batches sharded over ranks"), "model": "inception_v3", "global_batch": B * world,
                       "seq_len": None, "parallelism": f"dp{world}", "ranks": world, "hip_graph": use_graph,
                       "lanes": args.lanes,
                       "allreduce": (None if ar is None else
                                     {"transport": "jr_comm (RCCL)" if ar.comm is not None else
                                      f"torch.distributed {dist.get_backend()}", "buckets": len(ar.buckets),
                                      "payload": ar.payload, "fenced_issue_points_per_step": ar.fences,
                                      "world": world,
                                      "issue_point_ready_ms_vs_backward_end": overlap}),
                       "tiles": eng.tiles,
                       "conv_math": CONV_MATH[args.conv_math] if args.dtype == "f32" else "bf16 MFMA"},
            ("final_loss" if train else "mean_prediction"): round(loss, 5),
            "rehearsal": rehearsal,
            "roofline": roof,
            "hbm_families": hbm,
        }
        if not args.no_cpu_baseline and world == 1 and train:
            log("cpu baseline")
            out["cpu_baseline"] = cpu_baseline(args, res)
        emit(json_fd, out)
    if dist:
        dist.barrier()
        if comm is not None:
            torch.cuda.synchronize()
            comm.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
