#!/bin/bash
# Round-6 measurement of the bench default (fp32, JR_F32_X6H convs): the
# driver's command line, a rocprofv3 kernel-trace summary of the same run
# shape, the PMC passes for `traffic`, and the bf16 line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; out=gpurun_out/meas; mkdir -p $out
timeout -k 10 400 python bench.py > $out/f32_line.json 2> $out/f32_line.log || exit 1
cat $out/f32_line.json
timeout -k 10 300 python bench.py --dtype bf16 --no-cpu-baseline > $out/bf16_line.json 2> $out/bf16_line.log || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/prof -o run --output-format csv -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/$out/prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/prof1 -o run --output-format csv -- \
  python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --lanes 1 > $R/$out/prof1.log 2>&1 || exit 1
cd $R
cp $(find $out/prof -name 'run_kernel_stats.csv' | head -1) $out/f32_kernel_stats.csv
f=$(find $out/prof1 -name 'run_kernel_trace.csv' | head -1)
python tools/conv_table.py $f 64 400 30 $out/f32_1lane_kernel_stats.csv 3 > $out/f32_step_breakdown.txt
rm -rf $out/prof/*/*/run_kernel_trace.csv $out/prof1
timeout -k 10 900 tools/pmc_step.sh f32 r06_f32x6h x6h || exit 1
cp gpurun_out/r06_f32x6h_pmc.json $out/
echo done
