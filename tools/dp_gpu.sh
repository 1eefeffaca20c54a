#!/bin/bash
# The DP step on one GPU: the plain step vs the step
# through jr.dist.BucketAllReduce over a world-1 RCCL group (torch transport
# and libjr's own communicator), interleaved, fp32 and bf16; then a
# rocprofv3 kernel trace of the DP step for tools/dp_overlap.py.
# usage (GPU box): tools/dp_gpu.sh [rounds] [steps]
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
rounds=${1:-2}; steps=${2:-100}
out=gpurun_out/dp
mkdir -p $out
for r in $(seq 1 $rounds); do
  for dt in f32 bf16; do
    for dp in off torch jr joineach; do
      a="--dp off"; env=""
      [ $dp = torch ] && a="--dp on --dp-transport torch"
      [ $dp = jr ] && a="--dp on --dp-transport jr"
      [ $dp = joineach ] && a="--dp on --dp-transport torch" && env="JR_DP_JOIN_EACH=1"
      env $env timeout -k 10 240 python bench.py --steps $steps --warmup 10 --no-cpu-baseline --no-roofline --dtype $dt $a \
        > $out/line_${dt}_${dp}_$r.json 2> $out/line_${dt}_${dp}_$r.log
      python -c "import json;d=json.load(open('$out/line_${dt}_${dp}_$r.json'));print('$dt $dp round $r', d['ms_per_step'], 'ms', d['config'].get('allreduce'))"
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for dt in bf16 f32; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/prof_$dt -o run --output-format csv -- \
    python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --dtype $dt --dp on \
    > $R/$out/prof_$dt.log 2>&1
  f=$(find $R/$out/prof_$dt -name 'run_kernel_trace.csv' | head -1)
  python3 $R/tools/dp_overlap.py $f 3 > $R/$out/overlap_$dt.txt
  cat $R/$out/overlap_$dt.txt
done
