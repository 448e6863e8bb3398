#!/bin/bash
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD/yolo-series_amd:$PWD
for v in 241 244 248 245 252 253; do
  timeout -k 10 120 python -u scripts/check_variant.py $v yolov7 2 256 256 >> gpurun_out/p8x_check.log 2>&1
done
timeout -k 10 900 python -u scripts/tune_ops.py --cands 231,241,242,244,248,245,252,253 --rounds 3 --ops 20,22,23,26,29,84,85 --out gpurun_out/p8x_tune.json > gpurun_out/p8x_tune.txt 2>&1
