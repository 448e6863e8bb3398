#!/bin/bash
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD/yolo-series_amd:$PWD
timeout -k 10 120 python -u scripts/check_variant.py 233 yolov7 2 256 256 > gpurun_out/p8o_check.log 2>&1
timeout -k 10 120 python -u scripts/check_variant.py 233 yolov7 4 640 640 >> gpurun_out/p8o_check.log 2>&1
timeout -k 10 120 python -u scripts/check_variant.py 233 yolov7-tiny 3 320 448 >> gpurun_out/p8o_check.log 2>&1
timeout -k 10 600 python -u scripts/tune_ops.py --cands 231,233 --rounds 3 --ops 3,8,10,12,17,19,20,21,22,26,29,36,49,50,59,84,85 --out gpurun_out/p8o_tune.json > gpurun_out/p8o_tune.txt 2>&1
