#!/bin/bash
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD/yolo-series_amd:$PWD
for v in 234 235 236; do
  timeout -k 10 120 python -u scripts/check_variant.py $v yolov7 2 256 256 >> gpurun_out/ws1_check.log 2>&1
  timeout -k 10 120 python -u scripts/check_variant.py $v yolov7 4 640 640 >> gpurun_out/ws1_check.log 2>&1
  timeout -k 10 120 python -u scripts/check_variant.py $v yolov7-tiny 3 320 448 >> gpurun_out/ws1_check.log 2>&1
done
timeout -k 10 600 python -u scripts/tune_ops.py --cands 234,235,236 --rounds 3 --ops 3,8,10,12,56,58,59,64,66,75,39,47 --out gpurun_out/ws1_tune.json > gpurun_out/ws1_tune.txt 2>&1
