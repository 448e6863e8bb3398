#!/bin/bash
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD/yolo-series_amd:$PWD
for v in 17 18 19; do timeout -k 10 120 python -u scripts/check_variant.py $v yolov7 2 256 256 >> gpurun_out/ws64x_check.log 2>&1; done
timeout -k 10 600 python -u scripts/tune_ops.py --cands 17,18,19 --rounds 3 --ops 1,4,5 --out gpurun_out/ws64x_tune.json > gpurun_out/ws64x_tune.txt 2>&1
