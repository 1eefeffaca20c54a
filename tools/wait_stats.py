"""Cross-lane synchronisation of one training step's call list: producer
waits (jr.lanes pwaits) and producer records, by consumer / producer kind and
by phase (a backward call waiting for a forward producer, ...).
python tools/wait_stats.py [f32|bf16] [batch] [res]"""
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jama16-retina-replication_amd"))
from jr.engine import Engine  # noqa: E402

dt = sys.argv[1] if len(sys.argv) > 1 else "bf16"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
res = int(sys.argv[3]) if len(sys.argv) > 3 else 299
e = Engine(B, res, res, dtype=dt, seed=0)
fwd, bwd, opt, _, _ = e._build_calls(B)
phase = {}
for name, lst in (("fwd", fwd), ("bwd", bwd), ("opt", opt)):
    for c in lst:
        if c.idx >= 0:
            phase[c.idx] = name
seq = sorted([c for c in fwd + bwd + opt if c.idx >= 0], key=lambda c: c.idx)
pw = [(c, seq[j]) for c in seq for _, j in c.pwaits]
print(f"{dt}: {len(seq)} calls, {len(pw)} producer waits, {sum(c.record for c in seq)} records, "
      f"{sum(len(c.waits) for c in seq)} tail waits")
cnt = Counter((phase[c.idx], phase[p.idx]) for c, p in pw)
print("by (consumer phase, producer phase):", dict(cnt))
cnt = Counter((c.name, p.name, phase[c.idx], phase[p.idx]) for c, p in pw)
for k, v in cnt.most_common(30):
    print(f"  {v:4d}  {k[0]:18s} <- {k[1]:18s} ({k[2]} <- {k[3]})")
if "-v" in sys.argv:
    for c in seq:
        def why(c, p):
            r = (set(c.reads) | set(c.writes)) & set(p.writes) | (set(c.writes) & set(p.reads))
            return "/".join(str(k) for k in sorted(r, key=str))[:60]
        w = ",".join(f"{seq[j].name}@{lj}#{j}[{why(c, seq[j])}]" for lj, j in c.pwaits)
        print(f"{c.idx:4d} L{c.lane} {phase[c.idx]} {c.name:18s} {'REC' if c.record else '   '} {('<- ' + w) if w else ''}")
