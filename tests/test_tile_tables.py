"""The committed MI355X conv tile tables (jr/tiles_mi355x.json, written by
tools/make_tile_tables.py on the GPU box; Engine(tiles="pinned"), train.py
--tiles pinned, bench.py --tiles pinned): every BASELINE workload has one,
every launch of that workload's plan is covered, and every config id names a
tile of the current libjr tables (jr_conv2d_num_configs) -- a stale table
after a kernel-table change fails here, on the CPU."""
import json
import os

import pytest

from conftest import PKG

TABLES = os.path.join(PKG, "jr", "tiles_mi355x.json")
CDT = {"x8": 2, "x8p": 3, "f32": 0, "bf16": 1, "x6h": 4}
WANT = {("x8", 64, 299, True), ("bf16", 64, 299, True), ("x8", 32, 299, False), ("bf16", 32, 299, False),
        ("bf16", 64, 587, True), ("x6h", 64, 299, True)}


def _tables():
    with open(TABLES) as f:
        return json.load(f)["tables"]


def test_every_baseline_workload_is_pinned():
    have = {(t["conv_math"], t["batch"], t["height"], t["train"]) for t in _tables()}
    assert WANT <= have, WANT - have


def test_tables_cover_the_plan_and_name_existing_tiles():
    from jr import _ffi
    from jr.inception import build_inception_v3
    from jr.plan import build_plan
    L = _ffi.load()
    for t in _tables():
        plan = build_plan(build_inception_v3(t["height"], t["width"]), True)
        names = {u.name for u in plan.units}
        assert set(t["configs"]) == names, (t["conv_math"], t["batch"], t["height"])
        ntiles = L.jr_conv2d_num_configs(CDT[t["conv_math"]])
        assert ntiles > 0
        for name, (f, wg, dg) in t["configs"].items():
            ids = [f] + ([wg] + list(dg) if t["train"] else [])
            for c in ids:
                if c < 0:
                    continue            # no override recorded: planner heuristic
                assert (c & 0xFF) < ntiles and 0 <= (c >> 8) < 4096, (name, c)   # tile index, split-K factor


def test_engine_lookup_finds_the_table():
    from jr.engine import pinned_tile_table
    t = pinned_tile_table("x8", 64, 299, 299, True)
    assert t is not None and t["batch"] == 64
    assert pinned_tile_table("x8", 63, 299, 299, True) is None
