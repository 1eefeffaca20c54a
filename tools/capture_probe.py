"""Probe: capture a multi-lane engine step into a HIP graph, raw
(jr_graph_begin/end) or through torch.cuda.CUDAGraph; run in a child per
variant so a crash names the variant."""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jama16-retina-replication_amd"))
if len(sys.argv) > 1:
    import numpy as np, torch, ctypes
    from jr.engine import Engine
    from jr import synth, _ffi
    mode, lanes = sys.argv[1], int(sys.argv[2])
    e = Engine(2, 107, 107, seed=3, lanes=lanes)
    e.set_batch(synth.fundus_batch(0, 2, 107), np.array([[1.0], [0.0]], np.float32))
    e.train_step(); e.synchronize()
    fwd, bwd, opt, _, ev = e._build_calls(2)
    torch.cuda.synchronize()
    if mode == "raw":
        e.capture()
        e.replay(); e.synchronize()
    else:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=e.stream):
            e._fork(); e._run(fwd); e._join(); e._run(bwd); e._join(); e._run(opt)
        g.replay(); torch.cuda.synchronize()
    print(mode, lanes, "ok loss", e.loss_value(), flush=True)
    sys.exit(0)
for mode in ("raw",):
    for lanes in (2, 3, 4):
        r = subprocess.run([sys.executable, __file__, mode, str(lanes)], capture_output=True, text=True, timeout=300)
        print(mode, lanes, "rc", r.returncode, r.stdout.strip()[-200:], r.stderr.strip()[-300:] if r.returncode else "", flush=True)
