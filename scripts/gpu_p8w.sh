#!/bin/bash
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD/yolo-series_amd:$PWD
timeout -k 10 120 python -u scripts/check_variant.py 238 yolov7 2 256 256 > gpurun_out/p8w_check.log 2>&1
timeout -k 10 120 python -u scripts/check_variant.py 238 yolov7 4 640 640 >> gpurun_out/p8w_check.log 2>&1
timeout -k 10 120 python -u scripts/check_variant.py 238 yolov7-tiny 3 320 448 >> gpurun_out/p8w_check.log 2>&1
timeout -k 10 200 python -u scripts/check_variant.py 238 yolov7 32 640 640 >> gpurun_out/p8w_check.log 2>&1
timeout -k 10 600 python -u scripts/tune_ops.py --cands 238 --rounds 3 --ops 2,3,10,11,13,14,15,16,51,52,58,60,64,66,67,69 --out gpurun_out/p8w_tune.json > gpurun_out/p8w_tune.txt 2>&1
