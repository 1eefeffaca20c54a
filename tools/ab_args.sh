#!/bin/bash
# Interleaved A/B of bench.py argument sets on one box (no roofline / CPU
# baseline), `rounds` times, ms/step per run.
# usage (on the GPU box): tools/ab_args.sh <rounds> "<common args>" "<args A>" "<args B>" ...
cd "$(dirname "$0")/.." || exit 1
rounds=$1; common=$2; shift 2
for r in $(seq 1 "$rounds"); do
  for a in "$@"; do
    out=$(timeout -k 10 150 python bench.py --no-roofline --no-cpu-baseline $common $a 2>&1)
    rc=$?
    ms=$(echo "$out" | grep -o '"ms_per_step": [0-9.]*' | head -1 | grep -o '[0-9.]*$')
    echo "round $r  [$a]  ms/step $ms"
    if [ $rc -ne 0 ]; then echo "$out" | tail -20; echo "rc=$rc, stopping"; exit $rc; fi
  done
done
