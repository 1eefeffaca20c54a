#!/bin/bash
# Sweep every tile x split-K of a set of layers (tools/conv_sweep.py), one
# process per (dtype, op, layer), each under its own time limit; stops at the
# first step that faults or times out (no further GPU work after that).
# usage (GPU box): tools/sweep_layers.sh <out> "<dtypes>" "<ops>" "<layers>" [reps]
out=$1; dts=$2; ops=$3; layers=$4; reps=${5:-10}
cd "$(dirname "$0")/.." || exit 1
mkdir -p "$(dirname "$out")"
: > "$out"
for dt in $dts; do for op in $ops; do for l in $layers; do
  timeout -k 10 150 python -u tools/conv_sweep.py $dt $op $l $reps >> "$out" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "sweep dt=$dt op=$op $l rc=$rc" >> "$out"; [ $rc -ne 1 ] && exit $rc; fi
done; done; done
