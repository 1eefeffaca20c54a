#!/bin/bash
# Interleaved A/B of two pinned tile tables (the committed jr/tiles_mi355x.json
# vs an alternative file), bench.py ms/step.  Runs on the GPU box's scratch copy.
# usage: tools/table_ab.sh <rounds> <alt.json> "<bench args>"
cd "$(dirname "$0")/.." || exit 1
J=jama16-retina-replication_amd/jr/tiles_mi355x.json
cp "$J" /tmp/tiles_new.json
for r in $(seq 1 "$1"); do
  for v in alt new; do
    if [ $v = alt ]; then cp "$2" "$J"; else cp /tmp/tiles_new.json "$J"; fi
    out=$(timeout -k 10 150 python bench.py --no-roofline --no-cpu-baseline $3 2>&1); rc=$?
    echo "round $r $v $(echo "$out" | grep -o '"ms_per_step": [0-9.]*' | head -1)"
    if [ $rc -ne 0 ]; then echo "$out" | tail -5; cp /tmp/tiles_new.json "$J"; exit $rc; fi
  done
done
cp /tmp/tiles_new.json "$J"
