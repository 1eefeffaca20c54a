#!/bin/bash
# Stream-K logical blocks by XCD: the stream-K tests on the new build, then
# same-box A/Bs of the pre-fma_mix build (libjr_prev), the fma_mix build
# (libjr_fm) and the current one, fp32 x6h and bf16.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; out=gpurun_out/skxcd; mkdir -p $out
J=jama16-retina-replication_amd/jr
timeout -k 10 600 python -u -m pytest tests/test_gpu_streamk.py tests/test_gpu_lanes299.py -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
tools/ab_lib.sh 2 100 "" $J/libjr_prev.so $J/libjr_fm.so $J/libjr.so || exit 1
tools/ab_lib.sh 2 100 "--dtype bf16" $J/libjr_fm.so $J/libjr.so || exit 1
