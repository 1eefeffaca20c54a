set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for dt in bf16 f32; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof2_$dt -o run --output-format csv -- \
  python3 $R/bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-roofline --dtype $dt > $R/gpurun_out/prof2_$dt.log 2>&1
f=$(find $R/gpurun_out/prof2_$dt -name 'run_kernel_trace.csv' | head -1)
python3 $R/tools/busy_union.py $f 4 > $R/gpurun_out/busy_$dt.txt
cp $(find $R/gpurun_out/prof2_$dt -name 'run_kernel_stats.csv' | head -1) $R/gpurun_out/r02c_${dt}_kernel_stats.csv
rm -f $f
done
