"""Drop-in for the reference's train.py: same flags, constants, printed lines,
checkpoints and operating-point CSV; the graph/session machinery is replaced
by jr (libjr HIP kernels on MI355X).

  python train.py [-t TRAIN_DIR] [-v VAL_DIR] [-sm SAVE_MODEL_PATH]
                  [-ss SAVE_SUMMARIES_DIR] [-so SAVE_OPERATING_THRESHOLDS_PATH]
                  [-sgd]
Multi-GPU (data parallel, RCCL): torchrun --nproc-per-node N train.py ...
Reference behaviour kept: BN uses batch statistics in
training and validation (Q1); weights start from Keras default init (Q2);
images are channels_last (Q3: the reference's channels_first path is a
reshape that scrambles pixels, so it is not reproduced).
"""
import argparse
import csv
import os
import random
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import lib.dataset  # noqa: E402
import lib.evaluation  # noqa: E402
import lib.metrics  # noqa: E402

# train.py:19-24
DEFAULT_TRAIN_DIR = "./data/eyepacs/bin2/train"
DEFAULT_VAL_DIR = "./data/eyepacs/bin2/validation"
DEFAULT_SAVE_MODEL_PATH = "./tmp/model"
DEFAULT_SAVE_SUMMARIES_DIR = "./tmp/logs"
DEFAULT_SAVE_OPERATING_THRESHOLDS_PATH = "./tmp/op_pts.csv"

# train.py:66-89
NUM_CHANNELS = 3
NUM_WORKERS = 8
LEARNING_RATE = 3e-3
MOMENTUM = 0.9
USE_NESTEROV = True
TRAIN_BATCH_SIZE = 64
NUM_EPOCHS = 200
WAIT_EPOCHS = 10
MIN_DELTA_AUC = 0.01
VAL_BATCH_SIZE = 64
NUM_THRESHOLDS = 200
KEPSILON = 1e-7
SHUFFLE_BUFFER_SIZE = 2048


def build_parser():
    p = argparse.ArgumentParser(
        description="Trains and saves neural network for detection of diabetic retinopathy.")
    p.add_argument("-t", "--train_dir", default=DEFAULT_TRAIN_DIR,
                   help="path to folder that contains training tfrecords")
    p.add_argument("-v", "--val_dir", default=DEFAULT_VAL_DIR,
                   help="path to folder that contains validation tfrecords")
    p.add_argument("-sm", "--save_model_path", default=DEFAULT_SAVE_MODEL_PATH,
                   help="path to where graph model should be saved")
    p.add_argument("-ss", "--save_summaries_dir", default=DEFAULT_SAVE_SUMMARIES_DIR,
                   help="path to folder where summaries should be saved")
    p.add_argument("-so", "--save_operating_thresholds_path", default=DEFAULT_SAVE_OPERATING_THRESHOLDS_PATH,
                   help="path to where operating points should be saved")
    p.add_argument("-sgd", "--vanilla_sgd", action="store_true",
                   help="use vanilla stochastic gradient descent instead of "
                        "nesterov accelerated gradient descent")
    # extras (not in the reference): resolution, epochs, seeds, device
    p.add_argument("--image_size", type=int, default=299, help="input resolution (299; 587 high-res variant)")
    p.add_argument("--num_epochs", type=int, default=NUM_EPOCHS)
    p.add_argument("--seed", type=int, default=0, help="weight init seed (ensemble member index)")
    p.add_argument("--dtype", default="f32", choices=["f32", "bf16"],
                   help="activation storage and conv arithmetic: f32 (the reference's; default) or bf16 MFMA "
                        "(BASELINE configs 3 and 5; parameters, gradients, momentum and BN statistics stay fp32)")
    p.add_argument("--conv_math", default="x6h", choices=["x8", "x8p", "x6h", "f32"],
                   help="fp32 convolution arithmetic (--dtype f32): x6h = power-of-two-scaled 3-way fp16 split, six "
                        "products on the matrix cores (fp32-accurate, default), x8 = exact 3-way bf16 split, eight "
                        "products, x8p = x8 on pre-split operand planes, f32 = fp32 MFMA")
    p.add_argument("--replica_dump_dir", default=None,
                   help="(data parallel check) every rank writes its parameters after each epoch as "
                        "<dir>/params_e<epoch>_r<rank>.npy (Keras layout, fp32)")
    p.add_argument("--tiles", default="pinned", choices=["pinned", "heuristic", "autotune"],
                   help="conv tile configs: pinned (default; the committed MI355X table of this workload, "
                        "jr/tiles_mi355x.json, else the heuristic), heuristic (a function of the layer shapes only) "
                        "-- with either, two runs on any MI355X sum in the same order and train bitwise-equal -- or "
                        "autotune (timed on rank 0 at start, broadcast to every rank); the table in use is saved in "
                        "the checkpoint .meta")
    p.add_argument("--tile_table", default=None,
                   help="checkpoint path (or JSON file) whose saved tile table to reuse: reproduces that run's "
                        "summation order exactly")
    p.add_argument("--shuffle_seed", type=int, default=None)
    p.add_argument("--max_steps_per_epoch", type=int, default=None)
    return p


def status_line(epoch, num_epochs, batch_num, xent, i_step=None):
    """train.py:191-203: one \\r-terminated status line."""
    width = len(str(num_epochs))
    parts = [f"Epoch: {epoch:>{width}}/{num_epochs:>{width}}", f"Batch: {batch_num:>4}, Xent: {xent:6.4}"]
    if i_step is not None:
        parts.append(f"Step: {i_step:>10}")
    return ", ".join(parts)


def load_tile_table(path: str) -> dict:
    """A saved tile table: from a checkpoint's .meta (jr.checkpoint) or a
    JSON file holding the table itself."""
    import json
    from jr import checkpoint
    if path.endswith(".json"):
        with open(path) as f:
            return json.load(f)
    meta = checkpoint.read_meta(path)
    if "tile_table" not in meta:
        raise ValueError(f"{path}: checkpoint carries no tile table")
    return meta["tile_table"]


def main(argv=None):
    args = build_parser().parse_args(argv)
    import torch
    from jr import checkpoint
    from jr.engine import Engine
    from jr.session import Session
    from jr.summary import FileWriter

    random.seed(432)                       # train.py:17

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if rank == 0:       # one copy of the reference's header lines, whatever the rank count
        print(f"Numpy version: {np.__version__}")
        print(f"Torch version: {torch.__version__} (libjr / MI355X backend)")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs for the N > 1 path on a one-GPU box (as evaluate.py's
    # and bench.py's): JR_ONE_DEVICE=1 puts every rank on cuda:0,
    # JR_DIST_BACKEND=gloo replaces RCCL (which refuses two ranks on one device)
    if os.environ.get("JR_ONE_DEVICE") == "1" or os.environ.get("JR_BENCH_ONE_DEVICE") == "1":
        local = 0
    backend = os.environ.get("JR_DIST_BACKEND", "nccl")
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    # small host-side collectives (seed, metric sums, replica digests) run on
    # device tensors under RCCL, host tensors under gloo
    coll_dev = "cuda" if backend == "nccl" else "cpu"

    if rank == 0:
        print(f"""
Training images folder: {args.train_dir},
Validation images folder: {args.val_dir},
Saving model and graph checkpoints at: {args.save_model_path},
Saving summaries at: {args.save_summaries_dir},
Saving operating points at: {args.save_operating_thresholds_path},
Use SGD: {bool(args.vanilla_sgd)}
""")

    thresholds = lib.metrics.generate_thresholds(NUM_THRESHOLDS, KEPSILON) + [0.5]
    size = [args.image_size, args.image_size]
    shuffle_seed = args.shuffle_seed if args.shuffle_seed is not None else int.from_bytes(os.urandom(4), "little")
    if dist:   # every rank walks the same shuffled stream of record handles
        t = torch.tensor([shuffle_seed], dtype=torch.int64, device=coll_dev)
        dist.broadcast(t, 0)
        shuffle_seed = int(t.item())
    # data parallel: each rank decodes only its own batches (b % world ==
    # rank) of the common stream; validation and the final sweep likewise,
    # with the metric counts summed over ranks (Session.sync_metrics)
    shard = (rank, world) if dist else None
    train_dataset = lib.dataset.initialize_dataset(
        args.train_dir, TRAIN_BATCH_SIZE, num_workers=NUM_WORKERS,
        prefetch_buffer_size=2 * TRAIN_BATCH_SIZE, shuffle_buffer_size=SHUFFLE_BUFFER_SIZE,
        image_data_format="channels_last", num_channels=NUM_CHANNELS, image_dim=size,
        seed=shuffle_seed, decode_dtype="uint8", shard=shard)
    val_dataset = lib.dataset.initialize_dataset(
        args.val_dir, VAL_BATCH_SIZE, num_workers=NUM_WORKERS,
        prefetch_buffer_size=2 * TRAIN_BATCH_SIZE, shuffle_buffer_size=SHUFFLE_BUFFER_SIZE,
        image_data_format="channels_last", num_channels=NUM_CHANNELS, image_dim=size,
        seed=shuffle_seed + 1, decode_dtype="uint8", shard=shard)

    engine = Engine(max(TRAIN_BATCH_SIZE, VAL_BATCH_SIZE), args.image_size, args.image_size,
                    device=local, optimizer="sgd" if args.vanilla_sgd else ("nesterov" if USE_NESTEROV else "momentum"),
                    lr=LEARNING_RATE, momentum=MOMENTUM, seed=args.seed, dtype=args.dtype,
                    conv_math=args.conv_math if args.dtype == "f32" else "bf16",
                    tiles="pinned" if args.tiles == "pinned" else "heuristic")
    table = None
    if args.tile_table:
        table = load_tile_table(args.tile_table)
    elif args.tiles == "autotune" and rank == 0:
        engine.autotune()
        table = engine.tile_table()
    if dist and args.tiles == "autotune" and not args.tile_table:
        box = [table]
        dist.broadcast_object_list(box, 0)
        table = box[0]
    if table is not None:
        engine.set_tile_table(table)
    sess = Session(engine, thresholds, NUM_THRESHOLDS, KEPSILON)
    sess.rank = rank
    if dist:
        from jr.dist import BucketAllReduce
        sess.allreduce = BucketAllReduce(engine, world)

        def _sum_over_ranks(vec):
            t = torch.from_numpy(vec).to(coll_dev)
            dist.all_reduce(t)
            return t.cpu().numpy()
        sess.reduce = _sum_over_ranks

    def check_replicas(epoch):
        """Data parallel: every rank applies the same update to the same
        reduced gradient, so the replicas must stay bitwise identical; compare
        a digest of every rank's parameters once per epoch (and dump them for
        --replica_dump_dir)."""
        if not dist and not args.replica_dump_dir:
            return
        flat = engine.params_numpy()
        if args.replica_dump_dir:
            os.makedirs(args.replica_dump_dir, exist_ok=True)
            np.save(os.path.join(args.replica_dump_dir, f"params_e{epoch}_r{rank}.npy"), flat)
        if dist:
            import hashlib
            digest = hashlib.sha256(flat.tobytes()).hexdigest()
            got = [None] * world
            dist.all_gather_object(got, digest)
            if len(set(got)) != 1:
                raise RuntimeError(f"data-parallel replicas diverged after epoch {epoch}: {got}")
    train_writer = FileWriter(os.path.join(args.save_summaries_dir, "train")) if rank == 0 else None

    latest_peak_auc = 0.0
    waited_epochs = 0
    saved = False
    steps_per_epoch = None
    if dist:   # every rank runs the same number of steps (matching collectives)
        steps_per_epoch = -(-train_dataset.num_records() // TRAIN_BATCH_SIZE) // world
    for epoch in range(args.num_epochs):
        sess.reset("brier")
        batch_num = 0
        it = iter(train_dataset)
        try:
            for images, labels in it:
                if steps_per_epoch is not None and batch_num >= steps_per_epoch:
                    break
                if args.max_steps_per_epoch is not None and batch_num >= args.max_steps_per_epoch:
                    break
                i_global, xent, probs = sess.train_batch(images, labels)
                sess.update(labels, probs, "brier")
                if rank == 0:
                    print(status_line(epoch, args.num_epochs, batch_num, xent, i_global), end="\r")
                batch_num += 1
        finally:
            lib.dataset.close_iterator(it)
        sess.sync_metrics("brier")
        check_replicas(epoch)
        train_brier = sess.value("brier")
        if rank == 0:
            print("\nEnd of epoch {0}! (Brier: {1:8.6})".format(epoch, train_brier))

        # every rank gets the same val_auc (summed counts), so the early-stop
        # decisions below agree and the collectives stay matched
        val_auc = lib.evaluation.perform_test(sess=sess, init_op=val_dataset,
                                              summary_writer=train_writer, epoch=epoch)
        if val_auc < latest_peak_auc + MIN_DELTA_AUC:
            if WAIT_EPOCHS == waited_epochs:
                if rank == 0:
                    print("Stopped early at epoch {0} with saved peak auc {1:10.8}".format(epoch + 1, latest_peak_auc))
                break
            waited_epochs += 1
        else:
            latest_peak_auc = val_auc
            if rank == 0:
                print(f"New peak auc reached: {val_auc:10.8}")
                checkpoint.save(args.save_model_path, engine.g, engine.params_numpy(),
                                {"epoch": epoch, "val_auc": float(val_auc), "tile_table": engine.tile_table()})
            saved = True
            waited_epochs = 0

    # train.py:272-300: restore the best weights, sweep the training set,
    # write specificity/sensitivity per threshold.
    if dist:
        dist.barrier()
    if saved:
        flat, _ = checkpoint.load(args.save_model_path, engine.g)
        engine.load_params(flat)
    sess.reset("tp", "fp", "fn", "tn")
    it = iter(train_dataset)
    try:
        for images, labels in it:
            probs = sess.predict(images, labels)
            sess.update(labels, probs, "tp", "fp", "fn", "tn")
    finally:
        lib.dataset.close_iterator(it)
    sess.sync_metrics("tp", "fp", "fn", "tn")
    if rank == 0:
        os.makedirs(os.path.dirname(os.path.abspath(args.save_operating_thresholds_path)), exist_ok=True)
        spec, sens = sess.specificities(), sess.sensitivities()
        with open(args.save_operating_thresholds_path, "w") as f:
            w = csv.writer(f, delimiter=" ")
            w.writerow(["threshold", "specificity", "sensitivity"])
            for idx in range(NUM_THRESHOLDS):
                w.writerow(["{:0.4f}".format(v) for v in (thresholds[idx], spec[idx], sens[idx])])
    if train_writer:
        train_writer.close()
    if dist:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
