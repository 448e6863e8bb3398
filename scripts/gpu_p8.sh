#!/bin/bash
# 8-phase ring: correctness on every conv layer shape (forced), then per-layer timing vs the dispatch
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD/yolo-series_amd:$PWD
timeout -k 10 120 python -u scripts/check_variant.py 231 yolov7 2 256 256 > gpurun_out/p8_check.log 2>&1
timeout -k 10 120 python -u scripts/check_variant.py 231 yolov7 4 640 640 >> gpurun_out/p8_check.log 2>&1
timeout -k 10 120 python -u scripts/check_variant.py 231 yolov7-tiny 3 320 448 >> gpurun_out/p8_check.log 2>&1
timeout -k 10 600 python -u scripts/tune_ops.py --cands 231,201 --rounds 3 --ops ${P8_OPS:-8,17,20,22,23,24,25,26,29,36,49,55,73,77,83,84,85} --out gpurun_out/p8_tune.json > gpurun_out/p8_tune.txt 2>&1
