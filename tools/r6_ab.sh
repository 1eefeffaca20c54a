#!/bin/bash
# Interleaved bench A/B of conv-math variants on one box (fp32 299^2 B=64).
# usage (GPU box): tools/r6_ab.sh rounds steps variant...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; out=gpurun_out/ab; mkdir -p $out
rounds=$1; steps=$2; shift 2
for r in $(seq 1 $rounds); do
  for m in "$@"; do
    timeout -k 10 200 python bench.py --steps $steps --warmup 10 --no-cpu-baseline --no-roofline --conv-math $m \
      > $out/line_${m}_$r.json 2> $out/line_${m}_$r.log || exit 1
    python -c "import json;d=json.load(open('$out/line_${m}_$r.json'));print('$m round $r', d['ms_per_step'], 'ms', d['value'], 'img/s')"
  done
done
