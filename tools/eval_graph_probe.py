"""Eval forward (evaluate.py's per-batch model call): eager two-lane launches
vs HIP-graph replay of the same forward (Engine.capture, producer waits as
graph edges), same process, interleaved; host enqueue time of the eager
forward; and whether the two give the same predictions bitwise.
python tools/eval_graph_probe.py [f32|bf16] [batch] [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jama16-retina-replication_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from jr import synth  # noqa: E402
from jr.engine import Engine  # noqa: E402

dt = sys.argv[1] if len(sys.argv) > 1 else "bf16"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
K = int(sys.argv[3]) if len(sys.argv) > 3 else 100
e = Engine(B, 299, 299, dtype=dt, seed=0, train=False)
e.set_batch(synth.fundus_batch(0, B, 299), synth.labels(0, B))
for _ in range(5):
    e.forward()
p_eager = e.predictions()
e.capture()
for _ in range(3):
    e.replay()
p_graph = e.predictions()


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        fn()
    th = time.perf_counter()
    e.synchronize()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    return (t1 - t0) / K * 1e3, (th - t0) / K * 1e3


for r in range(3):
    a, ah = timed(e.forward)
    b, bh = timed(e.replay)
    print(f"{dt} B={B} round {r}: eager {a:.3f} ms/forward (host enqueue {ah:.3f}), "
          f"graph {b:.3f} ms/forward (host {bh:.3f})", flush=True)
print(f"graph == eager predictions: {bool(np.array_equal(p_eager, p_graph))}")
e.close()
