#!/bin/bash
# Interleaved A/B of two builds on one box: bench.py of each tree (a copy of
# another commit's package + bench.py under a directory of this tree), no
# roofline / CPU baseline.  usage: tools/ab_dirs.sh <rounds> "<bench args>" <dir A> <dir B> ...
cd "$(dirname "$0")/.." || exit 1
rounds=$1; args=$2; shift 2
for r in $(seq 1 "$rounds"); do
  for d in "$@"; do
    out=$(cd "$d" && timeout -k 10 150 python bench.py --no-roofline --no-cpu-baseline $args 2>&1)
    rc=$?
    ms=$(echo "$out" | grep -o '"ms_per_step": [0-9.]*' | head -1 | grep -o '[0-9.]*$')
    echo "round $r  [$d]  ms/step $ms"
    if [ $rc -ne 0 ]; then echo "$out" | tail -20; echo "rc=$rc, stopping"; exit $rc; fi
  done
done
