"""Autotune the conv tiles of the BASELINE workloads once on an MI355X and
write them to jr/tiles_mi355x.json, the pinned tables Engine(tiles="pinned")
loads: every run on every MI355X then sums in the same order (bit-stable,
VERDICT r1 item 9) at autotuned speed.  Each workload is tuned REPS times in
fresh processes' worth of engines and the per-op majority kept (timing noise
between neighbours).  Regenerate whenever a tile table in
csrc/jr_conv_impl.h changes (tests/test_tile_tables.py checks every id is in
range of jr_conv2d_num_configs).

  python tools/make_tile_tables.py [out.json] [conv_math ...]     (GPU box)
With conv maths listed (e.g. bf16), only those workloads are re-tuned and the
other tables of the existing file are kept."""
import collections
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "jama16-retina-replication_amd"))

import torch  # noqa: E402

from jr.engine import Engine  # noqa: E402

# (dtype, conv_math, batch, res, train): BASELINE configs 2, 3, 4 (f32 / bf16 members), 5
WORKLOADS = [("f32", "x8", 64, 299, True), ("bf16", "bf16", 64, 299, True), ("f32", "x8", 32, 299, False),
             ("bf16", "bf16", 32, 299, False), ("bf16", "bf16", 64, 587, True), ("f32", "x8p", 64, 299, True),
             ("f32", "x6h", 64, 299, True), ("f32", "x6h", 32, 299, False)]
REPS = 3


def tune(dtype, math, B, res, train):
    eng = Engine(B, res, res, dtype=dtype, conv_math=math, train=train, autotune=False)
    eng.clear_tile_table()
    n = [0]

    def tick(name):     # a line every few units: the GPU box kills a run silent for 3 minutes
        n[0] += 1
        if n[0] % 8 == 0:
            print(f"    {math} B={B} {res}^2: unit {n[0]} {name}", flush=True)
    eng.autotune(progress=tick)
    t = eng.tile_table()
    t["train"] = train
    eng.clear_tile_table()
    del eng
    torch.cuda.empty_cache()
    return t


def main():
    default = os.path.join(ROOT, "jama16-retina-replication_amd", "jr", "tiles_mi355x.json")
    out = sys.argv[1] if len(sys.argv) > 1 else default
    # selectors: a conv math ("bf16") or one workload "math:batch:res:train" ("bf16:64:587:1")
    only = set(sys.argv[2:])
    sel = lambda w: (not only) or w[1] in only or f"{w[1]}:{w[2]}:{w[3]}:{int(w[4])}" in only  # noqa: E731
    key = lambda t: (t["conv_math"], t["batch"], t["height"], t["train"])  # noqa: E731
    tables = []
    if only:
        src = out if os.path.exists(out) else default   # resume into an existing output file
        with open(src) as f:
            tables = [t for t in json.load(f)["tables"]
                      if not any(sel(w) and key(t) == (w[1], w[2], w[3], w[4]) for w in WORKLOADS)]
    for w in WORKLOADS:
        if not sel(w):
            continue
        t0 = time.time()
        runs = []
        for r in range(REPS):
            runs.append(tune(*w))
            print(f"  {w} rep {r}: {time.time() - t0:.0f} s", flush=True)
        cfg = {}
        for name in runs[0]["configs"]:
            per = [r["configs"][name] for r in runs]
            f = collections.Counter(p[0] for p in per).most_common(1)[0][0]
            wg = collections.Counter(p[1] for p in per).most_common(1)[0][0]
            dg = [collections.Counter(p[2][i] for p in per).most_common(1)[0][0] for i in range(len(per[0][2]))]
            cfg[name] = [f, wg, dg]
        t = dict(runs[0])
        t["configs"] = cfg
        tables.append(t)
        print(f"{w}: {len(cfg)} launches tuned x{REPS} in {time.time() - t0:.0f} s", flush=True)
        with open(out, "w") as f:     # after every workload: a run cut short keeps what it finished
            json.dump({"device": torch.cuda.get_device_name(0), "tables": tables}, f, indent=1, sort_keys=True)
        print("wrote", out, flush=True)


if __name__ == "__main__":
    main()
