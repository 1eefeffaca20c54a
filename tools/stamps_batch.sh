set -e
for spec in "1 0 conv5 0" "1 0 conv5 5" "1 0 conv5 26" "1 0 c17x7 13" "1 0 c17x7 32" "1 0 m17 13" "1 0 m17 25" "3 0 conv5 9" "3 0 conv5 18" "3 0 c17x7 13" "1 2 conv5 26" "1 1 c17x7 13"; do
  timeout -k 10 60 python -u tools/conv_stamps.py $spec >> gpurun_out/stamps1.txt 2>&1
done
