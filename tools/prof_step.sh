#!/bin/bash
# rocprofv3 kernel-trace of a short bench run + per-step breakdown.
# usage (on the GPU box): tools/prof_step.sh <dtype> <tag> [lanes] [conv_math]
# (lanes 1 for the per-launch conv table: it maps GEMMs by issue order;
# --no-roofline: the family-rate replays after the timed steps would also
# launch the optimizer, which the table uses to delimit steps)
set -e
dt=$1; tag=$2; lanes=${3:-1}; math=${4:-f32}
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$tag -o run --output-format csv -- \
  python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --dtype $dt --lanes $lanes --conv-math $math > $R/gpurun_out/prof_$tag.log 2>&1
cd $R
f=$(find gpurun_out/prof_$tag -name 'run_kernel_trace.csv' | head -1)
python tools/conv_table.py $f 64 400 30 gpurun_out/${tag}_step_kernel_stats.csv 3 > gpurun_out/${tag}_step_breakdown.txt
cp $(find gpurun_out/prof_$tag -name 'run_kernel_stats.csv' | head -1) gpurun_out/${tag}_kernel_stats.csv
