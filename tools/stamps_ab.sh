#!/bin/bash
# A/B of two stamps builds on the same box: each spec runs under both
# libraries (JR_LIB_DIAG), alternating, each run under its own time limit.
# usage (GPU box): tools/stamps_ab.sh <out> <libA> <libB> "<spec>" ["<spec>" ...]
#   spec = "<dtype> <op> <layer> <cfg>"
out=$1; A=$2; B=$3; shift 3
cd "$(dirname "$0")/.." || exit 1
: > "$out"
for spec in "$@"; do
  for lib in "$A" "$B" "$A" "$B"; do
    echo "## $(basename $lib)" >> "$out"
    JR_LIB_DIAG=$lib timeout -k 10 60 python -u tools/conv_stamps.py $spec 3 >> "$out" 2>&1 || exit $?
  done
done
