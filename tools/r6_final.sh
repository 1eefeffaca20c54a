#!/bin/bash
# End-of-round evidence at the final build: pytest -m gpu, smoke(), the bench
# command's line (fp32 x6h default) and bf16, the rocprofv3 kernel-trace
# summary of the bench command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; out=gpurun_out/final; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; tail -3 $out/gpu_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -5 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
timeout -k 10 400 python bench.py > $out/f32x6h_line.json 2> $out/f32x6h_line.log || exit 1
cat $out/f32x6h_line.json
timeout -k 10 300 python bench.py --dtype bf16 --no-cpu-baseline > $out/bf16_line.json 2> $out/bf16_line.log || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/prof -o run --output-format csv -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/$out/prof.log 2>&1 || exit 1
cd $R; cp $(find $out/prof -name 'run_kernel_stats.csv' | head -1) $out/f32x6h_bench_kernel_stats.csv
rm -f $(find $out/prof -name 'run_kernel_trace.csv')
echo done
