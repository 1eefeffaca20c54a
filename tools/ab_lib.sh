#!/bin/bash
# Interleaved same-box A/B of two builds of libjr (JR_LIB), bench.py fp32
# x6h by default.  usage (GPU box): tools/ab_lib.sh rounds steps "<bench args>" libA libB ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; out=gpurun_out/ablib; mkdir -p $out
rounds=$1; steps=$2; args=$3; shift 3
for r in $(seq 1 $rounds); do
  for lib in "$@"; do
    t=$(basename $lib .so)
    JR_LIB=$R/$lib timeout -k 10 200 python bench.py --steps $steps --warmup 10 --no-cpu-baseline --no-roofline $args \
      > $out/line_${t}_$r.json 2> $out/line_${t}_$r.log || exit 1
    python -c "import json;d=json.load(open('$out/line_${t}_$r.json'));print('$t round $r', d['ms_per_step'], 'ms', d['value'], 'img/s')"
  done
done
