#!/bin/bash
# x8 convbench ablations after the split-shift fix (compare profiles/r03_convbench_x8.txt)
cd "$(dirname "$0")/.." || exit 1
timeout -k 10 200 python -u tools/convbench.py 0,11,13 x8 > gpurun_out/convbench_x8_r03b.txt 2>&1
