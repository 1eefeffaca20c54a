#!/bin/bash
# round-3 A/B/C of the bf16 conv loop changes (stamps builds); see DESIGN §3
cd "$(dirname "$0")/.." || exit 1
out=gpurun_out/stamps_abc.txt; : > $out
for spec in '1 0 conv5 5' '1 0 conv5 0' '1 0 c17x7 13' '1 2 c17x7 6' '1 2 c17x1 12' '1 0 c35x3 1' '1 1 c35x3 3' '1 0 m17 13' '3 0 c17x7 13' '3 0 conv5 9'; do
  for lib in jama16-retina-replication_amd/jr/libjr_stamps_base.so jama16-retina-replication_amd/jr/libjr_stamps_zp.so jama16-retina-replication_amd/jr/libjr_stamps.so jama16-retina-replication_amd/jr/libjr_stamps_base.so jama16-retina-replication_amd/jr/libjr_stamps_zp.so jama16-retina-replication_amd/jr/libjr_stamps.so; do
    echo "## $(basename $lib) $spec" >> $out
    JR_LIB_DIAG=$lib timeout -k 10 60 python -u tools/conv_stamps.py $spec 3 >> $out 2>&1 || exit $?
  done
done
for s in '2 0 conv5 11' '2 0 c17x7 11' '2 0 m17 13' '2 1 c17x7 11' '2 2 c17x7 11'; do
  JR_LIB_DIAG=jama16-retina-replication_amd/jr/libjr_stamps.so timeout -k 10 60 python -u tools/conv_stamps.py $s 3 >> gpurun_out/stamps_x8.txt 2>&1 || exit 1
done
