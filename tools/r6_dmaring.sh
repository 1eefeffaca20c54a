#!/bin/bash
# LDS-DMA from inline asm in the ring kernels (no compiler vmcnt(0) per
# stream-K K-tile): the whole GPU suite on the new build, then same-box A/Bs
# against the previous build (libjr_prev), fp32 x6h and bf16.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; out=gpurun_out/dmaring; mkdir -p $out
J=jama16-retina-replication_amd/jr
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; tail -3 $out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
tools/ab_lib.sh 2 100 "" $J/libjr_prev.so $J/libjr.so || exit 1
tools/ab_lib.sh 2 100 "--dtype bf16" $J/libjr_prev.so $J/libjr.so || exit 1
