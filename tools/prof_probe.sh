#!/bin/bash
# rocprofv3 --kernel-trace --stats of one probe command -> per-kernel summary.
# usage (on the GPU box): tools/prof_probe.sh <tag> <command...>
set -e
tag=$1; shift
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$tag -o run --output-format csv -- "$@" > $R/gpurun_out/prof_$tag.log 2>&1
f=$(find $R/gpurun_out/prof_$tag -name 'run_kernel_stats.csv' | head -1)
python3 - "$f" > $R/gpurun_out/${tag}_kstats.txt <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:70]:70s} calls {int(r['Calls']):5d}  avg {float(r['AverageNs']) / 1e3:9.1f} us  min {float(r['MinNs']) / 1e3:9.1f} us")
PY
rm -rf $R/gpurun_out/prof_$tag
