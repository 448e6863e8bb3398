#!/bin/bash
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD/yolo-series_amd:$PWD
timeout -k 10 120 python -u scripts/check_variant.py 0 yolov7 2 256 256 > gpurun_out/xcd_check.log 2>&1
timeout -k 10 120 python -u scripts/check_variant.py 0 yolov7 4 640 640 >> gpurun_out/xcd_check.log 2>&1
timeout -k 10 120 python -u scripts/check_variant.py 0 yolov7-tiny 3 320 448 >> gpurun_out/xcd_check.log 2>&1
timeout -k 10 600 python -u scripts/tune_ops.py --cands 255 --rounds 3 --ops 20,22,26,29,36,84,85 --out gpurun_out/xcd_tune.json > gpurun_out/xcd_tune.txt 2>&1
timeout -k 10 300 python -u scripts/op_profile.py --iters 4 --top 12 > gpurun_out/xcd_ops.txt 2>&1
bash scripts/pmc_traffic.sh
python3 scripts/pmc_traffic.py gpurun_out gpurun_out/xcd_pmc_traffic.json
