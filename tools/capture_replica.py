"""Replay the engine's real lane/wait schedule with tiny torch kernels in a
HIP graph capture: does the crash need libjr's kernels or only the pattern?
  python tools/capture_replica.py <lanes> <K> [libjr]"""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jama16-retina-replication_amd"))
if len(sys.argv) > 3:
    import numpy as np, torch
    from jr.engine import Engine
    from jr import synth
    lanes, K, mode = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    e = Engine(2, 107, 107, seed=3, lanes=lanes, autotune=False)
    e.set_batch(synth.fundus_batch(0, 2, 107), np.array([[1.0], [0.0]], np.float32))
    fwd, bwd, opt, _, _ = e._build_calls(2)
    seq = [c for c in fwd + bwd + opt if c.fn != "param_ready"][:K]
    bufs = [torch.zeros(4096, device="cuda") for _ in range(lanes)]
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=e.stream):
        e._fork()
        for c in seq:
            st = e.lane_streams[c.lane]
            for lj in c.waits:
                if mode.endswith("marker"):       # a fresh node on the waited lane
                    with torch.cuda.stream(e.lane_streams[lj]):
                        bufs[lj].add_(0)
                ev = torch.cuda.Event() if mode.endswith("fresh") else e._tail_ev[lj]
                ev.record(e.lane_streams[lj])
                st.wait_event(ev)
            if mode.startswith("torch"):
                with torch.cuda.stream(st):
                    bufs[c.lane].add_(1)
            else:
                rc = c.fn(*c.args)
                assert rc == 0, c.name
        e._join()
    g.replay()
    torch.cuda.synchronize()
    print("ok", mode, lanes, K)
    sys.exit(0)
for mode in ("torch_marker", "torch_fresh", "libjr_marker"):
    for K in (54, 10000):
        r = subprocess.run([sys.executable, __file__, sys.argv[1], str(K), mode], capture_output=True, text=True,
                           timeout=200)
        print(mode, K, "rc", r.returncode, r.stdout.strip()[-60:], flush=True)
