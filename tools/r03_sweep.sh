#!/bin/bash
# round 3: exhaustive tile x split-K sweeps of representative bf16 layers
# (tools/conv_sweep.py), one log per layer/op
cd "$(dirname "$0")/.." || exit 1
dt=${1:-1}
shift
for spec in "$@"; do
  set -- $spec
  timeout -k 10 150 python -u tools/conv_sweep.py $dt $2 $1 5 >> gpurun_out/sweep_dt${dt}.txt 2>&1 || exit $?
done
