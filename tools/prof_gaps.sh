#!/bin/bash
# rocprofv3 kernel trace of a short bench run -> where the step's wall time
# goes (tools/lane_profile.py) and where the GPU idles (tools/gap_profile.py).
# usage (on the GPU box): tools/prof_gaps.sh <tag> "<bench args>" ["ENV=.. ENV2=.."]
set -e
tag=$1; args=$2; envs=${3:-}
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && export TMPDIR=/tmp
[ -n "$envs" ] && export $envs
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_$tag -o run --output-format csv -- \
  python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline $args > $R/gpurun_out/prof_$tag.log 2>&1
cd $R/tools
f=$(find $R/gpurun_out/prof_$tag -name 'run_kernel_trace.csv' | head -1)
{ python lane_profile.py $f 3 30; echo; python gap_profile.py $f 3 30; } > $R/gpurun_out/${tag}_gaps.txt
rm -rf $R/gpurun_out/prof_$tag
