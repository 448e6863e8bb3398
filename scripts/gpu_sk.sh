#!/bin/bash
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD/yolo-series_amd:$PWD
timeout -k 10 120 python -u scripts/check_variant.py 237 yolov7 2 256 256 > gpurun_out/sk_check.log 2>&1
timeout -k 10 120 python -u scripts/check_variant.py 237 yolov7 4 640 640 >> gpurun_out/sk_check.log 2>&1
timeout -k 10 120 python -u scripts/check_variant.py 237 yolov7-tiny 3 320 448 >> gpurun_out/sk_check.log 2>&1
timeout -k 10 200 python -u scripts/check_variant.py 237 yolov7 32 640 640 >> gpurun_out/sk_check.log 2>&1
timeout -k 10 600 python -u scripts/tune_ops.py --cands 237 --rounds 3 --ops 20,22,23,26,29,36,49,77,84,85 --out gpurun_out/sk_tune.json > gpurun_out/sk_tune.txt 2>&1
