#!/bin/bash
# Re-judge round 5's two rejected faster fp32 variants against the calibrated
# fp32 curve bars: HEAD, the K-bounded filter-gradient
# split rule (JR_WGRAD_SPLIT_KMAX=80000) and the direct conv2d_1 kernel
# (JR_CONV1_DIRECT=1): the golden curve tests under each, then interleaved
# bench timings.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; out=gpurun_out/rejudge; mkdir -p $out
declare -A ENV=([head]="" [kmax]="JR_WGRAD_SPLIT_KMAX=80000" [conv1]="JR_CONV1_DIRECT=1")
for v in head kmax conv1; do
  env ${ENV[$v]} timeout -k 10 300 python -u -m pytest tests/test_gpu_golden.py -v -s --timeout 240 \
    --timeout-method thread -k "loss_curve_per_step_b16 and not bf16 or loss_curve_per_step_b4" > $out/curves_$v.log 2>&1
  echo "$v curves rc=$? $(grep -c PASSED $out/curves_$v.log) passed $(grep -c FAILED $out/curves_$v.log) failed"
  grep "fp32 population" $out/curves_$v.log
done
for r in 1 2 3; do
  for v in head kmax conv1; do
    env ${ENV[$v]} timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-roofline \
      > $out/line_${v}_$r.json 2> $out/line_${v}_$r.log || exit 1
    python -c "import json;d=json.load(open('$out/line_${v}_$r.json'));print('$v round $r', d['ms_per_step'], 'ms')"
  done
done
