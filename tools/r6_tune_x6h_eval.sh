#!/bin/bash
# The x6h eval tile table (B=32 forward, BASELINE config 4) autotuned x3, then
# the grouped ensemble (10 members, 4,096 images) A/B vs the x8-copy table.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; out=gpurun_out/tuneev; mkdir -p $out
cand=jama16-retina-replication_amd/jr/tiles_candidate_x6h_eval.json
timeout -k 10 600 python -u tools/make_tile_tables.py $cand x6h:32:299:0 > $out/tune.log 2>&1 || { tail -5 $out/tune.log; exit 1; }
tail -2 $out/tune.log; cp $cand $out/
for r in 1 2; do
  for t in copy tuned; do
    env $([ $t = tuned ] && echo JR_TILE_TABLES=$cand) timeout -k 10 300 python bench.py --mode ensemble --members 10 \
      --images 4096 --no-roofline > $out/ens_${t}_$r.json 2> $out/ens_${t}_$r.log || exit 1
    python -c "import json;d=json.load(open('$out/ens_${t}_$r.json'));print('$t round $r', d['value'], 'img/s', d['gpu_forward_only_images_per_s'], 'gpu-only')"
  done
done
