#!/bin/bash
# Interleaved A/B of libjr variants on one box: bench.py (no roofline / CPU
# baseline) for each library in turn, `rounds` times, ms/step per run.
# usage (on the GPU box): tools/ab_bench.sh <rounds> "<bench args>" lib1.so lib2.so ...
# (library paths relative to jama16-retina-replication_amd/jr/)
cd "$(dirname "$0")/.." || exit 1
rounds=$1; args=$2; shift 2
for r in $(seq 1 "$rounds"); do
  for lib in "$@"; do
    out=$(JR_LIB=jama16-retina-replication_amd/jr/$lib timeout -k 10 150 python bench.py --no-roofline --no-cpu-baseline $args 2>&1)
    rc=$?
    ms=$(echo "$out" | grep -o '"ms_per_step": [0-9.]*' | grep -o '[0-9.]*$')
    echo "round $r  $lib  ms/step $ms"
    if [ $rc -ne 0 ]; then echo "$out" | tail -20; echo "rc=$rc, stopping"; exit $rc; fi
  done
done
