#!/bin/bash
# rocprofv3 kernel stats + GPU-busy analysis of bench.py variants on one box.
# usage (on the GPU box): tools/prof_ab.sh <tag> "<bench args>" [<tag> "<bench args>" ...]
set -e
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
while [ $# -ge 2 ]; do
  tag=$1; args=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pab_$tag -o run --output-format csv -- \
    python3 $R/bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-roofline $args > $R/gpurun_out/pab_$tag.log 2>&1
  f=$(find $R/gpurun_out/pab_$tag -name 'run_kernel_trace.csv' | head -1)
  python3 $R/tools/busy_union.py $f 4 > $R/gpurun_out/pab_busy_$tag.txt
  python3 $R/tools/kernel_families.py $f 4 > $R/gpurun_out/pab_fam_$tag.txt
  rm -f $f
done
