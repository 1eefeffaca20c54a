"""Per-shape PMC table of the BN backward (tools/bn_pmc.sh passes over
tools/bn_pmc_run.py): for k_bn_reduce and k_bn_relu_bwd_apply of each BN
shape, the HBM-side bytes (FETCH_SIZE x 2 -- gfx950 tallies 128-B requests
at 64 B, MI355X_MICROARCH.md -- and WRITE_SIZE) against the kernel's own
algorithmic bytes, the L2 hit rate, the share of L2 misses that reached
DRAM (TCC_EA0_RDREQ_DRAM / TCC_EA0_RDREQ: the rest hit the Infinity Cache),
TA busy per active cycle, mean resident waves per CU, and the duration.
  python tools/bn_pmc_summary.py <dtype> <pass dir> ...   -> table on stdout"""
import csv
import glob
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from bnbench_shapes import SHAPES  # noqa: E402

esz = 2 if sys.argv[1] == "bf16" else 4
ctr = {}
names = {}
for d in sys.argv[2:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_bn_" not in r["Kernel_Name"]:
                continue
            did = int(r["Dispatch_Id"])
            names[(d, did)] = r["Kernel_Name"].split("(")[0].replace("void ", "")
            key = (d, did)
            ctr.setdefault(key, {})
            ctr[key][r["Counter_Name"]] = ctr[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            if "Start_Timestamp" in r and "End_Timestamp" in r:
                ctr[key]["_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
# per pass dir: the last 3 * len(SHAPES) BN dispatches, in order
per = {}
for d in sys.argv[2:]:
    ids = sorted(k for k in ctr if k[0] == d)[-3 * len(SHAPES):]
    per[d] = ids
rows = []
for s, (h, c, cnt) in enumerate(SHAPES):
    m = 64 * h * h
    for role, off, alg in (("reduce", 0, 2 * m * c * esz), ("apply", 2, 3 * m * c * esz)):
        v = {}
        kname = None
        for d, ids in per.items():
            if len(ids) < 3 * len(SHAPES):
                continue
            k = ids[3 * s + off]
            kname = names[k]
            for n, x in ctr[k].items():
                v.setdefault(n, x)
        fetch = 2 * v.get("FETCH_SIZE", 0) * 1024
        write = v.get("WRITE_SIZE", 0) * 1024
        hit, miss = v.get("TCC_HIT_sum", 0), v.get("TCC_MISS_sum", 0)
        rd, rdd = v.get("TCC_EA0_RDREQ_sum", 0), v.get("TCC_EA0_RDREQ_DRAM_sum", 0)
        gui = v.get("GRBM_GUI_ACTIVE", 0)
        rows.append({"shape": f"{h}^2x{c}", "layers": cnt, "kernel": kname, "role": role,
                     "alg_MB": round(alg / 1e6, 2), "hbm_side_MB": round((fetch + write) / 1e6, 2),
                     "ratio": round((fetch + write) / alg, 2) if alg else None,
                     "l2_hit": round(hit / (hit + miss), 3) if hit + miss else None,
                     "dram_share_of_l2_reads": round(rdd / rd, 3) if rd else None,
                     "ta_busy_per_cycle": round(v.get("TA_TA_BUSY_sum", 0) / gui, 2) if gui else None,
                     "waves_per_cu": round(v.get("SQ_LEVEL_WAVES", 0) / max(v.get("SQ_BUSY_CYCLES", 1), 1), 2),
                     "gui_cycles": gui})
print(json.dumps(rows, indent=1))
