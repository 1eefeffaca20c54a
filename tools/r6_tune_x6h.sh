#!/bin/bash
# Autotune the JR_F32_X6H tile table of the bench workload (x3, majority) into
# a candidate file, then A/B it against the x8-copy table, interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; out=gpurun_out/tune; mkdir -p $out
cand=jama16-retina-replication_amd/jr/tiles_candidate_x6h.json
timeout -k 10 900 python -u tools/make_tile_tables.py $cand x6h > $out/tune.log 2>&1 || { tail -5 $out/tune.log; exit 1; }
tail -3 $out/tune.log
cp $cand $out/tiles_candidate_x6h.json
for r in 1 2 3; do
  for t in copy tuned; do
    env $([ $t = tuned ] && echo JR_TILE_TABLES=$cand) timeout -k 10 200 python bench.py --steps 100 --warmup 10 \
      --no-cpu-baseline --no-roofline --conv-math x6h > $out/line_${t}_$r.json 2> $out/line_${t}_$r.log || exit 1
    python -c "import json;d=json.load(open('$out/line_${t}_$r.json'));print('$t round $r', d['ms_per_step'], 'ms')"
  done
done
