#!/bin/bash
# end of round 3: rocprofv3 --kernel-trace --stats of the driver's own bench
# command at HEAD, and the per-family kernel times of its trace
set -e
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r03f_drv -o run --output-format csv -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/prof_r03f_drv.log 2>&1
cd $R
cp $(find gpurun_out/prof_r03f_drv -name 'run_kernel_stats.csv' | head -1) gpurun_out/r03f_f32_bench_kernel_stats.csv
python tools/kernel_families.py $(find gpurun_out/prof_r03f_drv -name 'run_kernel_trace.csv' | head -1) > gpurun_out/r03f_f32_bench_families.txt 2>&1 || true
rm -rf gpurun_out/prof_r03f_drv/*/*_kernel_trace.csv.gz 2>/dev/null || true
