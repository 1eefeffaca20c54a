#!/bin/bash
# JR_F32_X6H in the grouped ensemble: the grouped / engine / config-4 tests,
# then the config-4 line (10 members x 57,000 images) with x6h, and a
# kernel trace of the two-lane bench for the gap profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; out=gpurun_out/ensx6h; mkdir -p $out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_ensemble.py tests/test_gpu_eval299.py -v -s --timeout 300 \
  --timeout-method thread > $out/tests.log 2>&1
rc=$?; echo "ensemble tests rc=$rc"; grep -E "FAILED|passed|failed|config 4" $out/tests.log | tail -12; ok $rc || exit $rc
timeout -k 10 560 python bench.py --mode ensemble --members 10 --images 57000 > $out/ens57k_f32x6h.json 2> $out/ens57k.log || exit 1
cat $out/ens57k_f32x6h.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $R/$out/prof -o run --output-format csv -- \
  python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $R/$out/prof.log 2>&1 || exit 1
cd $R; f=$(find $out/prof -name "run_kernel_trace.csv" | head -1)
python tools/gap_profile.py $f 3 25 > $out/gaps_f32x6h.txt; rm -f $f; head -40 $out/gaps_f32x6h.txt
