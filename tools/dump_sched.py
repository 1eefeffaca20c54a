import os, sys, json
sys.path.insert(0, "/root/repo/jama16-retina-replication_amd")
import numpy as np
from jr.engine import Engine
e = Engine(2, 107, 107, seed=3, lanes=3, autotune=False)
fwd, bwd, opt, _, _ = e._build_calls(2)
seq = [c for c in fwd + bwd + opt if c.fn != "param_ready"]
json.dump([(c.lane, c.waits, c.name) for c in seq], open("/root/repo/gpurun_out/sched3.json", "w"))
print(len(seq))
