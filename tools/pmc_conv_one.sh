#!/bin/bash
# PMC passes (one counter group per run) over tools/conv_one.py.
# usage (GPU box): tools/pmc_conv_one.sh <tag> <dtype> <op> <cfg> [layer]
set -e
tag=$1; shift
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && export TMPDIR=/tmp
i=0
for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $ctr -d $R/gpurun_out/pmc1_${tag}_$i -o run --output-format csv -- \
    python3 $R/tools/conv_one.py "$@" 5 > $R/gpurun_out/pmc1_${tag}_$i.log 2>&1
done
cd $R
python3 tools/pmc_one_summary.py gpurun_out/pmc1_${tag}_1 gpurun_out/pmc1_${tag}_2 gpurun_out/pmc1_${tag}_3 > gpurun_out/pmc1_${tag}.txt
rm -rf gpurun_out/pmc1_${tag}_1 gpurun_out/pmc1_${tag}_2 gpurun_out/pmc1_${tag}_3
