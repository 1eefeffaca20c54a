"""Input-pipeline throughput: lib.dataset.initialize_dataset over
a synthetic TFRecord of q=100 JPEG fundus images (the reference preprocess
writes JPEG q=100), images/s per num_workers.  CPU only.
  python tools/pipeline_bench.py [n_records] [workers,...]"""
import io
import os
import sys
import tempfile
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "jama16-retina-replication_amd"))

import numpy as np  # noqa: E402
from PIL import Image  # noqa: E402

from jr import synth, tfrecord  # noqa: E402
from lib.dataset import initialize_dataset  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    workers = [int(w) for w in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 4, 8, 16]
    imgs = synth.fundus_batch(0, 64, 299)
    jpgs = []
    for im in imgs:
        b = io.BytesIO()
        Image.fromarray(im).save(b, format="JPEG", quality=100)
        jpgs.append(b.getvalue())
    d = tempfile.mkdtemp(prefix="jr_pipe_")
    path = os.path.join(d, "train-00000.tfrecord")
    with tfrecord.TFRecordWriter(path) as w:
        for i in range(n):
            w.write(tfrecord.encode_example({"image/encoded": jpgs[i % 64], "image/format": b"jpeg",
                                             "image/class/label": i % 2, "image/height": 299, "image/width": 299}))
    print(f"{n} records, mean JPEG {np.mean([len(j) for j in jpgs]) / 1024:.0f} KiB, cpus {os.cpu_count()}")
    for nw in workers:
        for dtype in ("uint8", "float32"):
            ds = initialize_dataset(d, 64, num_workers=nw, prefetch_buffer_size=128, decode_dtype=dtype)
            t = time.perf_counter()
            cnt = sum(len(x) for x, _ in ds)
            dt = time.perf_counter() - t
            print(f"workers {nw:2d} {dtype:7s}: {cnt / dt:8.0f} img/s")
    os.remove(path)
    os.rmdir(d)


if __name__ == "__main__":
    main()
