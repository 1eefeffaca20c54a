"""Debug: per-conv forward outputs and dL/dy of jr.Engine vs the fp64 oracle."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jama16-retina-replication_amd"))
import numpy as np, torch
from jr.engine import Engine
from jr.init import unflatten
from jr import synth
from oracle.inception_ref import InceptionV3Ref

res = int(sys.argv[1]) if len(sys.argv) > 1 else 107
B = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dtype = sys.argv[3] if len(sys.argv) > 3 else "f32"
eng = Engine(B, res, res, seed=1, dtype=dtype, fuse_pool=False)   # every activation materialised
imgs = synth.fundus_batch(0, B, res)
y = synth.labels(0, B)
eng.set_batch(imgs, y)
ref = InceptionV3Ref(unflatten(eng.g, eng.params_numpy()), torch.float64)
ref.record = []
ref.train_step(imgs.astype(np.float32) * np.float32(1 / 255), y, {})
ref32 = InceptionV3Ref(unflatten(eng.g, eng.params_numpy()), torch.float32)
ref32.record = []
ref32.train_step(imgs.astype(np.float32) * np.float32(1 / 255), y, {})
eng.forward(); eng.backward(); eng.synchronize()
acts = [a.float().cpu().numpy() for a in eng.acts]
dacts = [None if d is None else d.float().cpu().numpy() for d in eng.dacts]
for n, yo, y32 in zip(eng.g.convs, ref.record, ref32.record):
    bf = eng.g.bufs[n.y.buf]
    a = acts[n.y.buf].reshape(B, bf.h, bf.w, bf.c)[..., n.y.c_off:n.y.c_off + n.cout]
    r = yo.detach().permute(0, 2, 3, 1).numpy()
    fe = np.max(np.abs(a - r)) / max(np.abs(r).max(), 1e-9)
    d = dacts[n.y.buf].reshape(B, bf.h, bf.w, bf.c)[..., n.y.c_off:n.y.c_off + n.cout]
    rg = yo.grad.permute(0, 2, 3, 1).numpy()
    ge = np.linalg.norm(d - rg) / max(np.linalg.norm(rg), 1e-30)
    r32 = y32.grad.permute(0, 2, 3, 1).double().numpy()
    ge32 = np.linalg.norm(r32 - rg) / max(np.linalg.norm(rg), 1e-30)
    fe32 = np.max(np.abs(y32.detach().permute(0, 2, 3, 1).double().numpy() - r)) / max(np.abs(r).max(), 1e-9)
    print(f"[cpu32 fwd {fe32:.2e} dy {ge32:.2e}] conv{n.idx+1:3d} {n.kh}x{n.kw}/{n.stride} {n.h}x{n.w}x{n.cin}->{n.cout} buf={bf.name}@{n.y.c_off} fwd_rel={fe:.2e} dy_rel={ge:.2e}")
