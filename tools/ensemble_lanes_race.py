"""what made the round-4 ensemble-lanes prototype give
different predictions on one and on two ranks (gpurun_out/t18.log).

The prototype ran jr.ensemble.EnsembleEngine's calls on two branch lanes
with ONE conv workspace for both.  Every grouped conv launch keeps its
split-K slabs, stream-K partial slots and BN-statistics partials in that
workspace, so two concurrent convs on different lanes overwrite each other's
partials.  This script runs the same batches through

  lanes=1                  (the default path),
  lanes=2, own workspaces  (the kept implementation: ("ws", lane) resources),
  lanes=2, shared          (lane 1's workspace replaced by lane 0's before
                            the call lists are bound: the prototype's layout),

and prints, per variant, whether every member's predictions are bitwise the
one-lane predictions.

  python tools/ensemble_lanes_race.py [--dtype f32] [--members 3] [--batches 6]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jama16-retina-replication_amd"))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--members", type=int, default=3)
    ap.add_argument("--batches", type=int, default=6)
    ap.add_argument("--res", type=int, default=299)
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    from jr import synth
    from jr.ensemble import EnsembleEngine
    from jr.inception import build_inception_v3
    from jr.init import init_params
    g = build_inception_v3(a.res, a.res)
    params = [init_params(g, m) for m in range(a.members)]
    xs = [synth.fundus_batch(1000 + 64 * k, a.batch, a.res) for k in range(a.batches)]

    def run(eng):
        out = []
        for x in xs:
            eng.set_batch(x)
            eng.forward()
            out.append(eng.predictions())
        return np.concatenate(out, axis=1)

    one = run(EnsembleEngine(params, a.batch, a.res, a.res, dtype=a.dtype, lanes=1))
    own = EnsembleEngine(params, a.batch, a.res, a.res, dtype=a.dtype, lanes=2)
    shared = EnsembleEngine(params, a.batch, a.res, a.res, dtype=a.dtype, lanes=2)
    shared.ws_lane[1] = shared.ws_lane[0]          # the prototype: one workspace for both lanes
    print(f"tiles {own.tiles}, {a.members} members, {a.batches} batches of {a.batch} at {a.res}^2, {a.dtype}")
    for name, eng in (("lanes=2, per-lane workspaces", own), ("lanes=2, ONE shared workspace", shared)):
        reps = [run(eng) for _ in range(3)]
        same = [bool(np.array_equal(r, one)) for r in reps]
        dev = max(float(np.abs(r - one).max()) for r in reps)
        print(f"{name}: bitwise equal to lanes=1 in {sum(same)}/3 passes, max |diff| {dev:.3e}")


if __name__ == "__main__":
    main()
