#!/bin/bash
# x8 (dtype 2) tile x split sweeps of the stem GEMMs, fp32-MFMA tiles (ids >= 14) included
# usage: tools/stem_sweep.sh "<op> <layer>" ...
cd "$(dirname "$0")/.." || exit 1
for spec in "$@"; do
  set -- $spec
  timeout -k 10 240 python tools/conv_sweep.py 2 $1 $2 5 2>&1 | grep -v amdgpu.ids | head -8 || exit 1
done
