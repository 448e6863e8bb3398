#!/bin/bash
# In-network sweep of the persistent-ring configurations (YV7_CONV_F16=2xx applies one to every conv
# that reaches the generic dispatch) on yolov7 640 bs32: per-op CSVs for a per-layer choice.
set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS:-201 202 205 206 213 215 216 217}; do
  YV7_CONV_F16=$v timeout -k 10 200 python scripts/op_profile.py --iters 5 --top 0 --csv gpurun_out/ops_v$v.csv > gpurun_out/op_v$v.txt 2>&1 || { echo "variant $v failed"; exit 1; }
done
echo done
