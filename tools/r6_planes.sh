#!/bin/bash
# (historical: ran at e0ab593; the planes path and JR_X6H_PLANES were removed after this A/B)
# x6h forward filters from pre-split planes: the bitwise test (planes vs the
# in-loop split), then an interleaved same-box A/B of JR_X6H_PLANES=0 / 1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; out=gpurun_out/planes; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_x6h_planes.py -v -x --timeout 300 --timeout-method thread > $out/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|Error|assert" $out/tests.log | head -20; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in 0 1; do
    JR_X6H_PLANES=$v timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-roofline \
      > $out/line_${v}_$r.json 2> $out/line_${v}_$r.log || exit 1
    python -c "import json;d=json.load(open('$out/line_${v}_$r.json'));print('planes=$v round $r', d['ms_per_step'], 'ms', d['value'], 'img/s')"
  done
done
