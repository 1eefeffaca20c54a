#!/bin/bash
# The fp32 schedule knobs re-checked for the x6h default (they were tuned on
# x8): interleaved bench rounds, one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; out=gpurun_out/knobs; mkdir -p $out
V=("default" "JR_WGRAD_SPLIT_TARGET=640" "JR_WGRAD_SPLIT_TARGET=512" "JR_WGRAD_SPLIT_TARGET=256" "JR_LANE_PRIORITY=0,0" "JR_DEFER_WGRAD=1" "JR_STEM_WGRAD_LANE=0")
for r in 1 2 3; do
  for i in "${!V[@]}"; do
    e=${V[$i]}; [ "$e" = default ] && e=""
    env $e timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-roofline \
      > $out/l_${i}_$r.json 2> $out/l_${i}_$r.log || exit 1
    python -c "import json;d=json.load(open('$out/l_${i}_$r.json'));print('${V[$i]}', 'round $r', d['ms_per_step'])"
  done
done
