"""Per-kernel averages of rocprofv3 --pmc passes (one counter group per pass
directory) with derived ratios:
  mfma_util   = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
                (MFMA busy cycles are summed over every SIMD; GRBM_GUI_ACTIVE
                is summed over the 8 XCDs: MI355X_MICROARCH.md, DVFS note)
  wait_frac   = SQ_WAIT_ANY / SQ_WAVE_CYCLES, issue_stall = SQ_WAIT_INST_ANY /
                SQ_WAVE_CYCLES, active = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  l2_hit      = TCC_HIT / (TCC_HIT + TCC_MISS)
  python tools/pmc_one_summary.py <pass dir> ... [--match substr]
"""
import csv
import glob
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--match=")), "k_conv")
acc = defaultdict(lambda: defaultdict(list))
for d in args:
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not files:
        print(f"# no counters in {d}")
        continue
    disp = {}
    for r in csv.DictReader(open(files[0])):
        if match not in r["Kernel_Name"]:
            continue
        e = disp.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "ctr": defaultdict(float)})
        e["ctr"][r["Counter_Name"]] += float(r["Counter_Value"])
    for e in disp.values():
        short = e["name"].split("(")[0].replace("void ", "")[:150]
        for k, v in e["ctr"].items():
            acc[short][k].append(v)
for name, ctr in acc.items():
    a = {k: sum(v) / len(v) for k, v in ctr.items()}
    print(name)
    for k in sorted(a):
        print(f"   {k:32s} {a[k]:.4g}   (n={len(ctr[k])})")
    der = {}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in a and a.get("GRBM_GUI_ACTIVE"):
        der["mfma_util"] = a["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * a["GRBM_GUI_ACTIVE"] / 8)
    if a.get("SQ_WAVE_CYCLES"):
        for k, n in (("SQ_WAIT_ANY", "wait_frac"), ("SQ_WAIT_INST_ANY", "issue_stall"),
                     ("SQ_ACTIVE_INST_ANY", "active"), ("SQ_WAIT_INST_LDS", "lds_issue_stall")):
            if k in a:
                der[n] = a[k] / a["SQ_WAVE_CYCLES"]
    if a.get("SQ_LDS_IDX_ACTIVE"):
        der["lds_conflict"] = a.get("SQ_LDS_BANK_CONFLICT", 0) / a["SQ_LDS_IDX_ACTIVE"]
    if "TCC_HIT_sum" in a:
        der["l2_hit"] = a["TCC_HIT_sum"] / max(a["TCC_HIT_sum"] + a["TCC_MISS_sum"], 1)
    for k, v in der.items():
        print(f"   => {k:29s} {v:.3f}")
