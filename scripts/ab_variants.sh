#!/bin/bash
# Per-op times of the yolov7-w6 1280 bs8 forward under each global conv variant (YV7_CONV_F16).
set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS:-2 6 7 8}; do
  YV7_CONV_F16=$v timeout -k 10 200 python scripts/op_profile.py --model yolov7-w6 --img 1280 --b 8 --iters 5 --top 0 --csv gpurun_out/ops_w6_v$v.csv > gpurun_out/op_w6_v$v.txt 2>&1 || exit 1
done
echo done
