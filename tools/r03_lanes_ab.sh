#!/bin/bash
# interleaved A/B of the lane count (eager launches), fp32 and bf16
cd "$(dirname "$0")/.." || exit 1
out=gpurun_out/lanes_ab_r03.txt; : > $out
for rep in 1 2; do
  for dt in f32 bf16; do
    for l in 2 3 4; do
      r=$(timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-roofline --dtype $dt --lanes $l 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])") || exit 1
      echo "rep $rep $dt lanes $l: $r ms/step" | tee -a $out
    done
  done
done
