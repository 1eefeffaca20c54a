#!/bin/bash
# JR_F32_X6H halo-tiled forward: the x6h op tests (halo ids included), then
# the bench workload's x6h table re-tuned with the halo ids as candidates,
# A/B against the committed x6h table, interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; out=gpurun_out/halo; mkdir -p $out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_x6h.py -v --timeout 300 --timeout-method thread > $out/ops.log 2>&1
rc=$?; echo "x6h op tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $out/ops.log | tail -12; ok $rc || exit $rc
[ $rc -eq 0 ] || exit 1
cand=jama16-retina-replication_amd/jr/tiles_candidate_halo.json
timeout -k 10 600 python -u tools/make_tile_tables.py $cand x6h:64:299:1 > $out/tune.log 2>&1 || { tail -5 $out/tune.log; exit 1; }
tail -2 $out/tune.log; cp $cand $out/
python - <<'PY'
import json
t=[t for t in json.load(open('jama16-retina-replication_amd/jr/tiles_candidate_halo.json'))['tables'] if t['conv_math']=='x6h' and t['train']][0]
h=[(k,v[0]) for k,v in t['configs'].items() if 42 <= (v[0] & 255) < 51]
print("halo picks:", len(h), h)
PY
for r in 1 2 3; do
  for t in committed halo; do
    env $([ $t = halo ] && echo JR_TILE_TABLES=$cand) timeout -k 10 200 python bench.py --steps 100 --warmup 10 \
      --no-cpu-baseline --no-roofline > $out/line_${t}_$r.json 2> $out/line_${t}_$r.log || exit 1
    python -c "import json;d=json.load(open('$out/line_${t}_$r.json'));print('$t round $r', d['ms_per_step'], 'ms')"
  done
done
