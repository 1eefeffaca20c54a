#!/bin/bash
# poolbench (per-shape pool kernel times) for each libjr variant, both dtypes
# usage: tools/pool_lib_ab.sh lib1.so lib2.so ...   (paths relative to jr/)
cd "$(dirname "$0")/.." || exit 1
for dt in bf16 f32; do
  for lib in "$@"; do
    echo "== $dt $lib"
    JR_LIB=jama16-retina-replication_amd/jr/$lib timeout -k 10 120 python tools/poolbench.py $dt | grep -E "avgpool|per step" || exit $?
  done
done
