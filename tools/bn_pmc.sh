#!/bin/bash
# rocprofv3 PMC passes over one BN backward launch set per BN shape
# (tools/bn_pmc_run.py), one counter group per run (MI355X_MICROARCH.md),
# summarised per shape by tools/bn_pmc_summary.py -> gpurun_out/bn_pmc_<dtype>.json
# usage (GPU box): tools/bn_pmc.sh <f32|bf16>
set -e
dt=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
i=0
dirs=""
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" \
           "SQ_LEVEL_WAVES SQ_BUSY_CYCLES SQ_WAVES TA_TA_BUSY_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d $R/gpurun_out/bnpmc_${dt}_$i -o run --output-format csv -- \
    python3 $R/tools/bn_pmc_run.py $dt > $R/gpurun_out/bnpmc_${dt}_$i.log 2>&1
  dirs="$dirs $R/gpurun_out/bnpmc_${dt}_$i"
done
cd $R
python tools/bn_pmc_summary.py $dt $dirs > gpurun_out/bn_pmc_${dt}.json
rm -rf $dirs
