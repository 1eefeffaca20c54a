#!/bin/bash
# A/B of HIP stream priorities per lane (JR_LANE_PRIORITY), bench.py ms/step
# usage: tools/prio_ab.sh <rounds> <dtype>
cd "$(dirname "$0")/.." || exit 1
for r in $(seq 1 "$1"); do
  for pr in "" "-1,0" "0,-1"; do
    out=$(JR_LANE_PRIORITY="$pr" timeout -k 10 150 python bench.py --no-roofline --no-cpu-baseline --dtype "$2" 2>&1); rc=$?
    echo "round $r $2 prio[${pr:-default}] $(echo "$out" | grep -o '"ms_per_step": [0-9.]*' | head -1)"
    if [ $rc -ne 0 ]; then echo "$out" | tail -5; exit $rc; fi
  done
done
