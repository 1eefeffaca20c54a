"""Is the host's enqueue loop ever the bound?  For the bench workload, times
(a) the host wall of enqueueing one training step while the GPU is still
busy with earlier steps (the Python call-list walk: ctypes calls + event
record / wait for the cross-lane dependencies), and (b) the GPU time per
step, over `steps` back-to-back steps.  Also counts the calls per step.

  python tools/host_probe.py [dtype] [steps]
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jama16-retina-replication_amd"))
import torch  # noqa: E402


def main():
    dtype = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    from jr import synth
    from jr.engine import Engine
    e = Engine(64, 299, 299, dtype=dtype, seed=0)
    e.set_batch(synth.fundus_batch(0, 64, 299), synth.labels(0, 64))
    for _ in range(3):
        e.train_step()
    e.synchronize()
    fwd, bwd, opt, _, _ = e._build_calls(64)
    n = sum(1 for c in fwd + bwd + opt if c.fn != "param_ready")
    waits = sum(len(c.waits) for c in fwd + bwd + opt if c.fn != "param_ready")
    # host time per step with the GPU several steps behind: enqueue `steps`
    # steps back to back; the GPU cannot be the bound of the enqueue unless
    # the HIP queue fills up, so host time per step is the walk's own cost
    t0 = time.perf_counter()
    host = []
    for _ in range(steps):
        a = time.perf_counter()
        e.train_step()
        host.append(time.perf_counter() - a)
    t_enq = time.perf_counter() - t0
    e.synchronize()
    t_all = time.perf_counter() - t0
    host.sort()
    print(f"{dtype}: {n} calls / step, {waits} cross-lane waits / step")
    print(f"host enqueue per step: median {host[len(host) // 2] * 1e3:.2f} ms, min {host[0] * 1e3:.2f} ms; "
          f"all {steps} steps enqueued in {t_enq * 1e3:.1f} ms, finished after {t_all * 1e3:.1f} ms "
          f"({t_all / steps * 1e3:.3f} ms per step on the GPU)")
    # per-call host cost of the bare ctypes path (a tiny kernel, no waits)
    c = next(c for c in opt if c.fn != "param_ready")
    a = time.perf_counter()
    for _ in range(200):
        c.fn(*c.args)
    b = time.perf_counter()
    e.synchronize()
    print(f"one optimizer call's host cost: {(b - a) / 200 * 1e6:.1f} us (ctypes + launch)")
    ev = torch.cuda.Event()
    a = time.perf_counter()
    for _ in range(200):
        ev.record(e.lane_streams[1])
        e.stream.wait_event(ev)
    b = time.perf_counter()
    print(f"one cross-lane wait (event record + wait): {(b - a) / 200 * 1e6:.1f} us")


if __name__ == "__main__":
    main()
