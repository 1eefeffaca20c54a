#!/bin/bash
# The x6h split on v_fma_mix_f32: the bitwise probe, the x6h op tests, then an
# interleaved bench A/B against x8 (whose split is unchanged).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; out=gpurun_out/fmamix; mkdir -p $out
timeout -k 10 120 tools/probes/fmamix_probe > $out/probe.txt 2>&1; rc=$?; cat $out/probe.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_gpu_x6h.py -q --timeout 300 --timeout-method thread > $out/ops.log 2>&1
rc=$?; tail -3 $out/ops.log; [ $rc -eq 0 ] || exit $rc
tools/r6_ab.sh ${1:-2} 100 x8 x6h
