#!/bin/bash
# rocprofv3 kernel trace of a short bench run -> per-family ms/step
# (tools/kernel_families.py over the last 3 whole steps).
# usage (on the GPU box): tools/prof_families.sh <tag> "<bench args>" ["ENV=.. ENV2=.."]
set -e
tag=$1; args=$2; envs=${3:-}
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && export TMPDIR=/tmp
[ -n "$envs" ] && export $envs
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$tag -o run --output-format csv -- \
  python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline $args > $R/gpurun_out/prof_$tag.log 2>&1
cd $R
f=$(find gpurun_out/prof_$tag -name 'run_kernel_trace.csv' | head -1)
python tools/kernel_families.py $f 3 > gpurun_out/${tag}_families.txt
cp $(find gpurun_out/prof_$tag -name 'run_kernel_stats.csv' | head -1) gpurun_out/${tag}_kernel_stats.csv
rm -rf gpurun_out/prof_$tag
