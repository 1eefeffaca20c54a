#!/bin/bash
# Interleaved A/B of environment settings on one box: bench.py (no roofline /
# CPU baseline) under each setting in turn, `rounds` times, ms/step per run.
# usage (on the GPU box): tools/ab_env.sh <rounds> "<bench args>" "A=1 B=2" "A=0" ...
cd "$(dirname "$0")/.." || exit 1
rounds=$1; args=$2; shift 2
for r in $(seq 1 "$rounds"); do
  for setting in "$@"; do
    out=$(env $setting timeout -k 10 150 python bench.py --no-roofline --no-cpu-baseline $args 2>&1)
    rc=$?
    ms=$(echo "$out" | grep -o '"ms_per_step": [0-9.]*' | grep -o '[0-9.]*$')
    echo "round $r  [$setting]  ms/step $ms"
    if [ $rc -ne 0 ]; then echo "$out" | tail -20; echo "rc=$rc, stopping"; exit $rc; fi
  done
done
