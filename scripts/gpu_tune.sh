#!/bin/bash
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD/yolo-series_amd:$PWD
timeout -k 10 1000 python -u scripts/tune_ops.py --out gpurun_out/tune_ops.json > gpurun_out/tune_ops.txt 2>&1
