"""Input-pipeline throughput (reference lib/dataset.py:5-59):
lib.dataset.initialize_dataset over a synthetic TFRecord of q=100 299^2 JPEG
fundus images (the reference preprocess writes JPEG q=100), run by N
concurrent rank processes, each with shard=(rank, N) -- i.e. what N
data-parallel ranks of train.py / evaluate.py do on one host.  Reports the
aggregate images/s (records all ranks delivered / wall time of the slowest
rank) per decoder (native libjr_jpeg vs Pillow) and per-rank worker count,
next to the CPU share this process may use (affinity, cgroup quota).

  python tools/pipeline_bench.py [--records N] [--ranks 1,8] [--workers 2,4]
                                 [--decoders native,pillow] [--dtype uint8]
CPU only."""
import argparse
import io
import multiprocessing as mp
import os
import sys
import tempfile
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "jama16-retina-replication_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def cpu_share():
    n = len(os.sched_getaffinity(0))
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(q) // int(p)))
    except (OSError, ValueError):
        pass
    return n


def _rank(rank, world, d, batch, workers, decoder, dtype, q):
    from lib.dataset import initialize_dataset
    ds = initialize_dataset(d, batch, num_workers=workers, prefetch_buffer_size=4 * batch, decode_dtype=dtype,
                            shard=(rank, world), jpeg_decoder=decoder)
    t = time.perf_counter()
    cnt = sum(len(x) for x, _ in ds)
    q.put((cnt, time.perf_counter() - t))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=4096)
    ap.add_argument("--ranks", default="1,8")
    ap.add_argument("--workers", default="2")
    ap.add_argument("--decoders", default="native,pillow")
    ap.add_argument("--dtype", default="uint8")
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    from PIL import Image
    from jr import synth, tfrecord
    from jr import jpeg as native_jpeg
    imgs = synth.fundus_batch(0, 64, 299)
    jpgs = []
    for im in imgs:
        b = io.BytesIO()
        Image.fromarray(im).save(b, format="JPEG", quality=100)
        jpgs.append(b.getvalue())
    d = tempfile.mkdtemp(prefix="jr_pipe_")
    path = os.path.join(d, "train-00000.tfrecord")
    with tfrecord.TFRecordWriter(path) as w:
        for i in range(a.records):
            w.write(tfrecord.encode_example({"image/encoded": jpgs[i % 64], "image/format": b"jpeg",
                                             "image/class/label": i % 2, "image/height": 299, "image/width": 299}))
    print(f"{a.records} records, mean JPEG {np.mean([len(j) for j in jpgs]) / 1024:.0f} KiB, "
          f"os.cpu_count {os.cpu_count()}, cpu share {cpu_share()}, native jpeg {native_jpeg.available()}", flush=True)
    ctx = mp.get_context("spawn")
    try:
        for dec in a.decoders.split(","):
            if dec == "native" and not native_jpeg.available():
                print("native: libjr_jpeg.so not built, skipped", flush=True)
                continue
            for world in (int(r) for r in a.ranks.split(",")):
                for nw in (int(w) for w in a.workers.split(",")):
                    q = ctx.Queue()
                    ps = [ctx.Process(target=_rank, args=(r, world, d, a.batch, nw, dec, a.dtype, q))
                          for r in range(world)]
                    for p in ps:
                        p.start()
                    res = [q.get(timeout=600) for _ in ps]
                    for p in ps:
                        p.join()
                    cnt = sum(c for c, _ in res)
                    wall = max(t for _, t in res)
                    print(f"decoder {dec:6s} ranks {world:2d} workers/rank {nw:2d} {a.dtype}: "
                          f"{cnt / wall:8.0f} img/s aggregate ({cnt} images, slowest rank {wall:.2f} s)", flush=True)
    finally:
        os.remove(path)
        os.rmdir(d)


if __name__ == "__main__":
    main()
