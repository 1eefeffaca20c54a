#!/bin/bash
# Interleaved A/B of HIP-graph replay vs eager launches (bench.py --no-graph), ms/step.
# usage (on the GPU box): tools/graph_ab.sh <rounds> <dtype>
cd "$(dirname "$0")/.." || exit 1
for r in $(seq 1 "$1"); do
  for args in "--graph" ""; do
    out=$(timeout -k 10 150 python bench.py --no-roofline --no-cpu-baseline --dtype "$2" $args 2>&1)
    rc=$?
    echo "round $r $2 [${args:-eager}] $(echo "$out" | grep -o '"ms_per_step": [0-9.]*' | head -1)"
    if [ $rc -ne 0 ]; then echo "$out" | tail -5; exit $rc; fi
  done
done
