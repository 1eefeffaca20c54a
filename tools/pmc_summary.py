"""Summarise rocprofv3 --pmc passes over the last training step (between
the last two optimizer dispatches): per kernel family, the HBM bytes
(FETCH_SIZE x 2: on gfx950 FETCH_SIZE tallies 128-B requests at 64 B, see
MI355X_MICROARCH.md; WRITE_SIZE as reported), the SQ cycle counters and the
MFMA utilisation (busy SIMD-cycles / all SIMD-cycles of the family's
dispatches, <= 1).
  python tools/pmc_summary.py <pass dir> ...   -> JSON on stdout"""
import csv, glob, json, sys
from collections import defaultdict


def family(name):
    n = name.split("(")[0].replace("void ", "").split("<")[0]
    if n in ("jr::k_conv", "jr::k_conv_bf16", "jr::k_splitk_reduce", "jr::k_splitk_reduce_stats", "jr::k_stats_finalize"):
        return "conv"
    return n


out = {"families": defaultdict(lambda: defaultdict(float)), "dispatches": {}}
for d in sys.argv[1:]:
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not files:
        continue
    rows = list(csv.DictReader(open(files[0])))
    disp = {}
    for r in rows:
        did = int(r["Dispatch_Id"])
        e = disp.setdefault(did, {"name": r["Kernel_Name"], "ctr": {}})
        e["ctr"][r["Counter_Name"]] = e["ctr"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(disp)
    opt = [i for i in ids if "k_nesterov" in disp[i]["name"] or "k_sgd" in disp[i]["name"]]
    if len(opt) < 2:
        continue
    window = [i for i in ids if opt[-2] < i <= opt[-1]]
    for i in window:
        f = family(disp[i]["name"])
        fam = out["families"][f]
        fam["dispatches_" + d.rsplit("_", 1)[-1]] += 1
        for k, v in disp[i]["ctr"].items():
            fam[k] += v
for f, c in out["families"].items():
    if "FETCH_SIZE" in c:
        c["hbm_read_bytes"] = 2 * c["FETCH_SIZE"] * 1024      # FETCH_SIZE is in KiB
    if "WRITE_SIZE" in c:
        c["hbm_write_bytes"] = c["WRITE_SIZE"] * 1024
    # MFMA utilisation: busy cycles summed over every SIMD (32 per
    # 32x32x16 bf16 MFMA) over the family's SIMD-cycles, i.e. 1024 SIMDs x
    # its dispatches' cycles (GRBM_GUI_ACTIVE is summed over the 8 XCDs)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c and c.get("GRBM_GUI_ACTIVE"):
        c["mfma_util"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * c["GRBM_GUI_ACTIVE"] / 8.0)

out["families"] = {k: dict(v) for k, v in out["families"].items()}
print(json.dumps(out, indent=1, sort_keys=True))
