#!/bin/bash
# round-3: bf16 loop before/after the incremental address walk (stamps builds)
cd "$(dirname "$0")/.." || exit 1
out=gpurun_out/stamps_ab2.txt; : > $out
for spec in '1 0 conv5 0' '1 0 conv5 5' '1 1 conv5 12' '1 2 conv5 26' '1 0 c35x5 3' '1 1 c35x5 3' '1 2 c35x5 3' '1 2 c17x7 6' '1 2 c17x1 12' '1 2 c8x1 6' '1 2 c35x3 6' '3 0 conv5 9'; do
  for lib in jama16-retina-replication_amd/jr/libjr_stamps_base.so jama16-retina-replication_amd/jr/libjr_stamps.so jama16-retina-replication_amd/jr/libjr_stamps_base.so jama16-retina-replication_amd/jr/libjr_stamps.so; do
    echo "## $(basename $lib) $spec" >> $out
    JR_LIB_DIAG=$lib timeout -k 10 60 python -u tools/conv_stamps.py $spec 3 >> $out 2>&1 || exit $?
  done
done
