#!/bin/bash
# JR_F32_X6H on the GPU: op tests, whole-step / curve / lanes tests, then an
# interleaved bench A/B against the x8 default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; out=gpurun_out/x6h; mkdir -p $out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }     # pass or test failure; anything else (fault, timeout) stops
timeout -k 10 500 python -u -m pytest tests/test_gpu_x6h.py -v -s --timeout 300 --timeout-method thread > $out/ops.log 2>&1
rc=$?; echo "x6h op tests rc=$rc"; grep -E "PASSED|FAILED|Error" $out/ops.log | tail -20; ok $rc || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_gpu_baseline_sizes.py tests/test_gpu_golden.py tests/test_gpu_lanes299.py \
  -k "x6h" -v -s --timeout 300 --timeout-method thread > $out/step.log 2>&1
rc=$?; echo "x6h step tests rc=$rc"; grep -E "PASSED|FAILED|population|gpu:" $out/step.log | cut -c1-400; ok $rc || exit $rc
for r in 1 2 3; do
  for m in x8 x6h; do
    timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-roofline --conv-math $m \
      > $out/line_${m}_$r.json 2> $out/line_${m}_$r.log || exit 1
    python -c "import json;d=json.load(open('$out/line_${m}_$r.json'));print('$m round $r', d['ms_per_step'], 'ms', d['value'], 'img/s')"
  done
done
