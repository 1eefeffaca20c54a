"""Eager two-lane steps vs HIP-graph replay of the same step (Engine.capture;
JR_GRAPH_PRECISE=1 captures the producer waits instead of tail waits), same
process, interleaved: ms per step each way.
python tools/graph_probe.py [f32|bf16] [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jama16-retina-replication_amd"))
import torch  # noqa: E402

from jr import synth  # noqa: E402
from jr.engine import Engine  # noqa: E402

dt = sys.argv[1] if len(sys.argv) > 1 else "bf16"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 40
e = Engine(64, 299, 299, dtype=dt, seed=0)
e.set_batch(synth.fundus_batch(0, 64, 299), synth.labels(0, 64))
for _ in range(3):
    e.train_step()
e.synchronize()
e.capture()
for _ in range(3):
    e.replay()
e.synchronize()


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        fn()
    e.synchronize()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / K * 1e3


for r in range(3):
    a = timed(e.train_step)
    b = timed(e.replay)
    print(f"round {r}: eager {a:.3f} ms/step, graph {b:.3f} ms/step ({os.environ.get('JR_GRAPH_PRECISE', '0')})",
          flush=True)
