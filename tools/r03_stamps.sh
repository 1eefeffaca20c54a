#!/bin/bash
# round 3: per-block stamps of representative conv GEMMs (stamps build) and
# the x8 ablation variants (tools/convbench.py)
cd "$(dirname "$0")/.." || exit 1
out=gpurun_out/stamps_r03.txt
for spec in "1 0 c17x7 13" "1 0 c17x7 38" "1 0 conv5 26" "1 0 conv5 5" "1 0 c17x1 13" "1 2 c17x7 3079" "1 1 c17x7 13" "1 0 m17 13" "2 0 conv5 11" "2 0 c17x7 11" "2 0 conv5 13" "2 1 c17x7 11"; do
  echo "## $spec" >> $out
  JR_LIB_DIAG=jama16-retina-replication_amd/jr/libjr_stamps.so timeout -k 10 60 python -u tools/conv_stamps.py $spec 3 >> $out 2>&1 || exit $?
done
timeout -k 10 200 python -u tools/convbench.py 0,11,13 x8 > gpurun_out/convbench_x8_r03.txt 2>&1
