#!/bin/bash
# Interleaved A/B of conv-math variants in the config-4 ensemble (10 members,
# 4,096 images, grouped launches): bench.py --mode ensemble.
# usage (GPU box): tools/r6_ab_ens.sh rounds variant...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; out=gpurun_out/abens; mkdir -p $out
rounds=$1; shift
for r in $(seq 1 $rounds); do
  for m in "$@"; do
    timeout -k 10 300 python bench.py --mode ensemble --members 10 --images 4096 --no-roofline --no-cpu-baseline \
      --conv-math $m > $out/ens_${m}_$r.json 2> $out/ens_${m}_$r.log || exit 1
    python -c "import json;d=json.load(open('$out/ens_${m}_$r.json'));print('$m round $r', d['value'], 'img/s', d['gpu_forward_only_images_per_s'], 'gpu-only')"
  done
done
