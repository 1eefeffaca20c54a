#!/bin/bash
# BASELINE config 4 at its stated size on one GPU: 10
# members x 57,000 synthetic test images, evaluate.predict_all end to end,
# bf16 and fp32 (x8); then the DP overlap line with the small tail bucket.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r6
for dt in ${ENS_DTYPES:-bf16 f32}; do
  timeout -k 10 560 python bench.py --mode ensemble --members 10 --images 57000 --dtype $dt \
    > gpurun_out/r6/ens57k_$dt.json 2> gpurun_out/r6/ens57k_$dt.log || exit 1
  cat gpurun_out/r6/ens57k_$dt.json
done
for dt in f32 bf16; do
  timeout -k 10 200 python bench.py --dp on --steps 50 --warmup 10 --no-cpu-baseline --no-roofline --dtype $dt \
    > gpurun_out/r6/dp_tail_$dt.json 2> gpurun_out/r6/dp_tail_$dt.log || exit 1
  cat gpurun_out/r6/dp_tail_$dt.json
done
