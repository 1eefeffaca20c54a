"""Drop-in for the reference's evaluate.py: same flags, model-path expansion
(comma list or glob), linear ensemble average, metrics, printed lines and
CSV; inference runs on libjr (MI355X).

  python evaluate.py (-e | -m | -o --data_dir D) [-lm PATHS] [-so CSV] [-b 32] [-op 0.5]
Multi-GPU: torchrun --nproc-per-node N evaluate.py ... shards whole batches
(dataset order, so every BN batch is the reference's, App. C Q1) across
ranks with no collective on the data path; rank 0 gathers the [N] per-model
predictions, averages and scores them.

The reference restores and runs one member at a time, re-reading and
re-decoding the test set per member (evaluate.py:166-211).  Here every
member is resident on the GPU at once (one engine each: parameters plus
batch-32 buffers, a few GB per member against 288 GB of HBM), and each test
batch is decoded once and run through all members -- the same batches, so
the same batch-statistics BN (App. C Q1) and the same predictions.
"""
import argparse
import csv
import os
import random
import sys
from glob import glob

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import lib.dataset  # noqa: E402
import lib.evaluation  # noqa: E402
import lib.metrics  # noqa: E402

# evaluate.py:24-29
DEFAULT_EYEPACS_DIR = "./data/eyepacs/bin2/test"
DEFAULT_MESSIDOR_DIR = "./data/messidor/bin2"
DEFAULT_LOAD_MODEL_PATH = "./tmp/model"
DEFAULT_SAVE_OPERATING_THRESHOLDS_PATH = "./tmp/test_op_pts.csv"
DEFAULT_BATCH_SIZE = 32

# evaluate.py:96-101
NUM_CHANNELS = 3
NUM_WORKERS = 8
NUM_THRESHOLDS = 200
KEPSILON = 1e-7


def build_parser():
    p = argparse.ArgumentParser(
        description="Evaluate performance of trained graph on test data set. "
                    "Specify --data_dir if you use the -o param.")
    p.add_argument("-m", "--messidor", action="store_true", help="evaluate performance on Messidor-Original")
    p.add_argument("-e", "--eyepacs", action="store_true", help="evaluate performance on EyePacs set")
    p.add_argument("-o", "--other", action="store_true", help="evaluate performance on your own dataset")
    p.add_argument("--data_dir", help="directory where data set resides")
    p.add_argument("-lm", "--load_model_path", default=DEFAULT_LOAD_MODEL_PATH,
                   help="path to where graph model should be loaded from creates an ensemble if paths are "
                        "comma separated or a regexp")
    p.add_argument("-so", "--save_operating_thresholds_path", default=DEFAULT_SAVE_OPERATING_THRESHOLDS_PATH,
                   help="path to where operating points metrics should be saved")
    p.add_argument("-b", "--batch_size", default=DEFAULT_BATCH_SIZE, help="batch size")
    p.add_argument("-op", "--operating_threshold", default=0.5, help="operating threshold")
    p.add_argument("--dtype", default="f32", choices=["f32", "bf16"],
                   help="activation storage and conv arithmetic: f32 (the reference's; default) or bf16 MFMA")
    p.add_argument("--conv_math", default="x6h", choices=["x8", "x8p", "x6h", "f32"],
                   help="fp32 convolution arithmetic: x6h = power-of-two-scaled 3-way fp16 split, six f16 MFMAs per "
                        "product (fp32-accurate, default: 8.5 %% faster than x8 on the 10-member ensemble, "
                        "profiles/r06_ab_ens_x8_x6h.txt), x8 = exact 3-way bf16 split, x8p = x8 on pre-split "
                        "operand planes, f32 = fp32 MFMA")
    p.add_argument("--per_member", action="store_true",
                   help="one engine per ensemble member (default: every member's layers in one grouped launch, "
                        "jr.ensemble; predictions are bitwise the same)")
    return p


def expand_model_paths(load_model_path: str):
    """evaluate.py:74-83: comma list, or glob when the path holds '*', '+'
    or '?' (each match's last extension stripped, duplicates removed).  Stems
    that are not complete checkpoints (a leftover `.data-*.tmp` of an
    interrupted save strips to `<path>.data-00000-of-00001`) are dropped."""
    from jr import checkpoint
    if "," in load_model_path:
        return load_model_path.split(",")
    if any(ch in load_model_path for ch in "*+?"):
        stems = {".".join(x.split(".")[:-1]) for x in glob("{}*".format(load_model_path))}
        return sorted(s for s in stems if checkpoint.exists(s))
    return [load_model_path]


def make_engines(paths, meta, batch_size, device=0, conv_math="x6h", dtype="f32", grouped=False):
    """The ensemble's inference engines, parameters loaded; conv tiles from
    the committed MI355X table of the eval workload (tiles="pinned"; the
    heuristic where none matches): every member and every run sums in the
    same order.  grouped: ONE jr.ensemble.EnsembleEngine holding every member
    (one launch per layer for all members); else one jr.Engine per member."""
    from jr import checkpoint
    from jr.engine import Engine
    if grouped and conv_math != "x8p":
        from jr.ensemble import EnsembleEngine
        params = [checkpoint.load(path, None)[0] for path in paths]
        return EnsembleEngine(params, batch_size, meta["height"], meta["width"], meta.get("units", 1), device=device,
                              dtype=dtype, conv_math=conv_math if dtype == "f32" else "bf16")
    engines = []
    for path in paths:
        eng = Engine(batch_size, meta["height"], meta["width"], meta.get("units", 1), device=device,
                     train=False, dtype=dtype, conv_math=conv_math if dtype == "f32" else "bf16")
        flat, _ = checkpoint.load(path, eng.g)
        eng.load_params(flat)
        engines.append(eng)
    return engines


def predict_all(engines, data_dir, batch_size, rank=0, world=1):
    """Per-member predictions over this rank's batches: ([M][n_r, 1], [n_r, 1],
    batch indices).  Each batch is decoded once (this rank's batches only)
    and run through every member."""
    import torch
    grouped = hasattr(engines, "members")      # jr.ensemble.EnsembleEngine
    g = engines.g if grouped else engines[0].g
    dataset = lib.dataset.initialize_dataset(
        data_dir, batch_size, num_workers=NUM_WORKERS, prefetch_buffer_size=2 * batch_size,
        image_data_format="channels_last", num_channels=NUM_CHANNELS,
        image_dim=[g.height, g.width], decode_dtype="uint8",
        shard=(rank, world))
    preds = [[] for _ in range(engines.members if grouped else len(engines))]
    got_y, ids = [], []
    it = iter(dataset)
    try:
        for k, (x, y) in enumerate(it):
            ids.append(k * world + rank)
            got_y.append(y)
            # every member's forward is enqueued before the first result is
            # read back (one host sync per batch, not per member), while the
            # decoder threads already work on the next batches
            if grouped:       # every member's layer in one launch
                n = engines.set_batch(x, y)
                engines.forward(n)
                for m, p in enumerate(engines.predictions(n)):
                    preds[m].append(p)
                continue
            # (the uint8 batch crosses PCIe once for all members)
            xd = torch.as_tensor(x).to(engines[0].device)
            torch.cuda.current_stream(engines[0].device).synchronize()
            n = 0
            for e in engines:
                n = e.set_batch(xd, y)
                e.forward(n)
            for m, e in enumerate(engines):
                preds[m].append(e.predictions(n))
    finally:
        lib.dataset.close_iterator(it)
    empty = np.zeros((0, 1), np.float32)
    preds = [np.vstack(p) if p else empty for p in preds]
    labels = np.vstack(got_y) if got_y else empty
    return preds, labels, ids


def _one_batch(x, y):
    """feed_dict_fn for lib.evaluation.perform_test: one batch, then the end
    of the pass (evaluate.py:114-118 feed_images)."""
    state = {"done": False}

    def feed():
        if state["done"]:
            raise StopIteration
        state["done"] = True
        return {"x": x, "y": y}
    return feed


def main(argv=None):
    parser = build_parser()
    args = parser.parse_args(argv)
    # evaluate.py:53-56 (chained comparison kept as is, App. C Q5)
    if bool(args.eyepacs) == bool(args.messidor) == bool(args.other):
        print("Can only evaluate one data set at once!")
        parser.print_help()
        return 2
    if args.data_dir is not None:
        data_dir = str(args.data_dir)
    elif args.eyepacs:
        data_dir = DEFAULT_EYEPACS_DIR
    elif args.messidor:
        data_dir = DEFAULT_MESSIDOR_DIR
    else:
        print("Please specify --data_dir.")
        parser.print_help()
        return 2

    import torch
    from jr import checkpoint

    load_model_paths = expand_model_paths(str(args.load_model_path))
    batch_size = int(args.batch_size)
    operating_threshold = float(args.operating_threshold)
    save_path = str(args.save_operating_thresholds_path)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs for the N > 1 path on a one-GPU box (as bench.py's):
    # JR_ONE_DEVICE=1 puts every rank on cuda:0, JR_DIST_BACKEND=gloo replaces
    # RCCL (which refuses two ranks on one device); the only collective here
    # is the final all_gather_object of the predictions
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

    random.seed(432)
    if rank == 0:       # one copy of the reference's header lines, whatever the rank count
        print(f"Numpy version: {np.__version__}")
        print(f"Torch version: {torch.__version__} (libjr / MI355X backend)")
        print("""
Evaluating: {},
Saving operating thresholds metrics at: {},
Using operating treshold: {},
""".format(data_dir, save_path, operating_threshold))
        print("Trying to load model(s):\n{}".format("\n".join(load_model_paths)))

    thresholds = lib.metrics.generate_thresholds(NUM_THRESHOLDS, KEPSILON) + [operating_threshold]
    meta = checkpoint.read_meta(load_model_paths[0])
    engines = make_engines(load_model_paths, meta, batch_size, device=local, conv_math=args.conv_math,
                           dtype=args.dtype, grouped=not args.per_member)
    preds, labels, order = predict_all(engines, data_dir, batch_size, rank, world)

    if dist:   # gather every rank's batches to rank 0, restore dataset order
        gathered = [None] * world
        dist.all_gather_object(gathered, (order, preds, labels))
        if rank != 0:
            dist.destroy_process_group()
            return 0
        pieces = []
        for o, p, y in gathered:
            sizes = np.cumsum([0] + [batch_size] * len(o))
            # the last batch may be partial
            if len(o) and y.shape[0] < sizes[-1]:
                sizes[-1] = y.shape[0]
            for k, bi in enumerate(o):
                pieces.append((bi, [m[sizes[k]:sizes[k + 1]] for m in p], y[sizes[k]:sizes[k + 1]]))
        pieces.sort(key=lambda t: t[0])
        preds = [np.vstack([pc[1][m] for pc in pieces]) for m in range(len(load_model_paths))]
        labels = np.vstack([pc[2] for pc in pieces])

    all_predictions = np.array(preds)
    avg_pred = np.mean(all_predictions, axis=0)          # evaluate.py:214-217
    all_y = labels

    names = {"tp": lib.metrics.true_positives_at_thresholds, "fp": lib.metrics.false_positives_at_thresholds,
             "fn": lib.metrics.false_negatives_at_thresholds, "tn": lib.metrics.true_negatives_at_thresholds}
    state = {k: lib.metrics.create_reset_metric(f, scope=k, thresholds=thresholds) for k, f in names.items()}
    state["brier"] = lib.metrics.create_reset_metric(lib.metrics.mean_squared_error, scope="brier")
    state["auc"] = lib.metrics.create_reset_metric(lib.metrics.auc, scope="auc")
    for value, update, reset in state.values():
        reset()
        update(all_y, avg_pred)
    tp, fp, fn, tn = (state[k][0]() for k in ("tp", "fp", "fn", "tn"))
    test_conf_matrix = lib.metrics.confusion_matrix(tp[-1], fp[-1], fn[-1], tn[-1])
    test_brier, test_auc = state["brier"][0](), state["auc"][0]()
    test_specificities = tn / (tn + fp + np.float32(KEPSILON))
    test_sensitivities = tp / (tp + fn + np.float32(KEPSILON))

    print(f"Brier score: {test_brier:6.4}, AUC: {test_auc:10.8}")
    print(f"Confusion matrix at operating threshold {operating_threshold:0.3f}")
    print(test_conf_matrix[0])
    print("Specificity: {0:0.4f}, Sensitivity: {1:0.4f} at Operating Threshold {2:0.4f}.".format(
        test_specificities[-1], test_sensitivities[-1], thresholds[-1]))
    os.makedirs(os.path.dirname(os.path.abspath(save_path)), exist_ok=True)
    with open(save_path, "w") as f:
        w = csv.writer(f, delimiter=" ")
        w.writerow(["threshold", "specificity", "sensitivity"])
        for idx in range(NUM_THRESHOLDS):
            w.writerow(["{:0.4f}".format(v) for v in (thresholds[idx], test_specificities[idx],
                                                       test_sensitivities[idx])])
    if dist:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
