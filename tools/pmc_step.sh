#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, as MI355X_MICROARCH.md's
# HBM/rocprofv3 section prescribes) over a short eager bench run; the
# summary of the last training step goes to gpurun_out/<tag>_pmc.json.
# usage (on the GPU box): tools/pmc_step.sh <dtype> <tag> [conv_math]
set -e
dt=$1; tag=$2; math=${3:-x8}
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && export TMPDIR=/tmp
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $ctr -d $R/gpurun_out/pmc_${tag}_$i -o run --output-format csv -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-graph --dtype $dt --conv-math $math \
    > $R/gpurun_out/pmc_${tag}_$i.log 2>&1
done
cd $R
python tools/pmc_summary.py gpurun_out/pmc_${tag}_1 gpurun_out/pmc_${tag}_2 gpurun_out/pmc_${tag}_3 > gpurun_out/${tag}_pmc.json
# the per-dispatch counter CSVs are large (autotuning dispatches included):
# keep only the summary (gpurun_out/ comes back only under 64 MiB)
rm -rf gpurun_out/pmc_${tag}_1 gpurun_out/pmc_${tag}_2 gpurun_out/pmc_${tag}_3
