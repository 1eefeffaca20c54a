"""Bisect which captured call makes a multi-lane HIP graph capture crash:
capture the first K calls of the step (+ a join) in a child process."""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jama16-retina-replication_amd"))
if len(sys.argv) > 2:
    import numpy as np, torch, ctypes
    from jr.engine import Engine
    from jr import synth, _ffi
    lanes, K = int(sys.argv[1]), int(sys.argv[2])
    e = Engine(2, 107, 107, seed=3, lanes=lanes, autotune=False)
    e.set_batch(synth.fundus_batch(0, 2, 107), np.array([[1.0], [0.0]], np.float32))
    fwd, bwd, opt, _, ev = e._build_calls(2)
    seq = [c for c in fwd + bwd + opt if c.fn != "param_ready"][:K]
    if len(sys.argv) > 3:
        for c in seq[-3:]:
            print(c.idx, c.name, "lane", c.lane, "waits lanes", c.waits)
    torch.cuda.synchronize()
    _ffi.check("b", e.lib.jr_graph_begin(e._s))
    e._fork(); e._run(seq); e._join()
    ex = ctypes.c_void_p()
    _ffi.check("e", e.lib.jr_graph_end(e._s, ctypes.byref(ex)))
    print("ok", K, flush=True)
    sys.exit(0)
lanes = int(sys.argv[1])
def ok(K):
    r = subprocess.run([sys.executable, __file__, str(lanes), str(K)], capture_output=True, text=True, timeout=120)
    return r.returncode == 0
lo, hi = 1, 700
if ok(hi):
    print("no crash up to", hi); sys.exit(0)
while hi - lo > 1:
    mid = (lo + hi) // 2
    if ok(mid): lo = mid
    else: hi = mid
print("first crashing K", hi, flush=True)
r = subprocess.run([sys.executable, __file__, str(lanes), str(hi), "v"], capture_output=True, text=True, timeout=120)
print(r.stdout)
r = subprocess.run([sys.executable, __file__, str(lanes), str(lo), "v"], capture_output=True, text=True, timeout=120)
print(r.stdout)
