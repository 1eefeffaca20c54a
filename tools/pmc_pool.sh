#!/bin/bash
# rocprofv3 PMC passes over tools/poolbench.py (one counter group per run):
# per pool kernel, HBM bytes (FETCH_SIZE / WRITE_SIZE, KiB) and SQ cycle
# counters, averaged per dispatch -> gpurun_out/pool_pmc.txt.
# usage (on the GPU box): tools/pmc_pool.sh [f32|bf16]
set -e
dt=${1:-f32}
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && export TMPDIR=/tmp
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  POOLBENCH_N=3 timeout -s KILL 90 rocprofv3 --pmc $ctr -d $R/gpurun_out/pmcpool_$i -o run --output-format csv -- \
    python3 $R/tools/poolbench.py $dt > $R/gpurun_out/pmcpool_$i.log 2>&1 || echo "pass $i ($ctr) failed: $?"
done
cd $R
python3 - <<'PY' > gpurun_out/pool_pmc.txt
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmcpool_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        grid = r.get("Grid_Size", r.get("Grid_Size_X", ""))
        acc[(k, grid)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (k, grid), cs in sorted(acc.items()):
    if "pool" not in k:
        continue
    print(k, "grid", grid, " ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(cs.items())))
PY
rm -rf gpurun_out/pmcpool_1 gpurun_out/pmcpool_2 gpurun_out/pmcpool_3 gpurun_out/pmcpool_4
