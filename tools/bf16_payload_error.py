"""How much a bf16 gradient payload costs at world 8.

RCCL sums a bf16 buffer in bf16: every partial sum of the ring
reduce-scatter is rounded to bf16 again, so the summed gradient of 8 ranks
carries its own rounding plus up to 7 roundings of the running sum.  This
emulates exactly that on real Inception-v3 gradients: 8 ranks' fp32
gradients from the CPU restatement (oracle/inception_ref.py, fp32, 299^2,
one batch of B images per rank, Keras init seed 0), summed

  exact : fp64 sum,
  fp32  : fp32 ring (rank r0 first, 7 fp32 adds; RCCL's ring order per chunk),
  bf16  : each rank's gradient rounded to bf16, 7 bf16-rounded ring adds,

and reports the relative error of the fp32 / bf16 sums per parameter tensor
(norm of the difference / norm of the exact sum), against the envelope a
bf16 ENGINE itself has on the same gradients (the emulated-bf16 oracle's
per-tensor gradient norm gap to fp64 in tests/golden/net_res299_b64.npz).
  python tools/bf16_payload_error.py [B] > profiles/r03_bf16_payload_error.txt"""
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "jama16-retina-replication_amd"))


def bf16(x):
    """Round-to-nearest-even fp32 -> bf16 (returned as fp32)."""
    import torch
    return torch.as_tensor(np.asarray(x, np.float32)).to(torch.bfloat16).float().numpy()


def ring_sum(parts, rnd, world):
    """RCCL ring order: the flat buffer is cut into `world` chunks; chunk c's
    running sum starts at rank (c + 1) % world and visits the ranks in ring
    order, rounding every partial sum with `rnd`."""
    n = parts[0].size
    out = np.empty(n, np.float32)
    bounds = np.linspace(0, n, world + 1).astype(np.int64)
    for c in range(world):
        lo, hi = bounds[c], bounds[c + 1]
        r0 = (c + 1) % world
        s = rnd(parts[r0][lo:hi])
        for k in range(1, world):
            s = rnd(s + rnd(parts[(r0 + k) % world][lo:hi]))
        out[lo:hi] = s
    return out


def main():
    import torch
    from jr import synth
    from jr.inception import build_inception_v3
    from jr.init import init_params, unflatten
    from oracle.inception_ref import InceptionV3Ref
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    world = 8
    torch.set_num_threads(os.cpu_count() or 8)
    g = build_inception_v3(299, 299)
    P = unflatten(g, init_params(g, 0))
    names = sorted(P)
    parts = []
    t0 = time.time()
    for r in range(world):
        ref = InceptionV3Ref(P, torch.float32)
        x = synth.fundus_batch(r * B, B, 299).astype(np.float32) * np.float32(1 / 255)
        y = synth.labels(r * B, B)
        _, _, grads = ref.train_step(x, y, {})
        parts.append(np.concatenate([np.asarray(grads[k], np.float32).ravel() for k in names]))
    sizes = [np.asarray(P[k]).size for k in names]
    offs = np.cumsum([0] + sizes)
    exact = np.sum(np.stack(parts).astype(np.float64), axis=0)
    f32 = ring_sum(parts, lambda a: np.asarray(a, np.float32), world)
    b16 = ring_sum(parts, bf16, world)
    rel = {}
    for tag, s in (("fp32", f32), ("bf16", b16)):
        e = []
        for i, k in enumerate(names):
            lo, hi = offs[i], offs[i + 1]
            den = np.linalg.norm(exact[lo:hi])
            if den > 0:
                e.append(np.linalg.norm(s[lo:hi] - exact[lo:hi]) / den)
        rel[tag] = np.array(e)
    gold = np.load(os.path.join(ROOT, "tests", "golden", "net_res299_b64.npz"))
    env = np.abs(gold["grad_norms_bf16emu"] - gold["grad_norms"]) / np.maximum(gold["grad_norms"], 1e-30)
    projenv = np.abs(gold["grad_proj_bf16emu"] - gold["grad_proj"]) / np.maximum(np.abs(gold["grad_proj"]), 1e-30)
    print(f"# 8-rank gradient sum, per-rank batch {B} at 299^2 (fp32 CPU restatement, seed 0), "
          f"{len(names)} tensors, {time.time() - t0:.0f} s")
    for tag in ("fp32", "bf16"):
        r = rel[tag]
        print(f"{tag} payload ring sum: relative error per tensor median {np.median(r):.3e}  "
              f"p90 {np.percentile(r, 90):.3e}  max {r.max():.3e}")
    print(f"bf16 engine envelope (emulated-bf16 oracle vs fp64, 299^2 B=64): per-tensor |grad norm| gap "
          f"median {np.median(env):.3e} max {env.max():.3e}; Rademacher projection gap median "
          f"{np.median(projenv):.3e}")
    ratio = np.median(rel["bf16"]) / np.median(env)
    print(f"bf16 payload error / bf16 engine envelope (medians): {ratio:.3e} -> "
          f"{'bf16 payload inside the bf16 step envelope' if ratio < 0.1 else 'use the fp32 payload'}")


if __name__ == "__main__":
    main()
