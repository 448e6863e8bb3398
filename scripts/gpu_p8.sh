#!/bin/bash
# 8-phase ring: correctness on every conv layer shape (forced), then per-layer timing vs the dispatch
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD/yolo-series_amd:$PWD
timeout -k 10 120 python -u scripts/check_variant.py 231 yolov7 2 256 256 > gpurun_out/p8_check.log 2>&1
timeout -k 10 120 python -u scripts/check_variant.py 231 yolov7 4 640 640 >> gpurun_out/p8_check.log 2>&1
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_variants.py -k "every_conv" > gpurun_out/p8_tests.log 2>&1
timeout -k 10 600 python -u scripts/tune_ops.py --cands 231,201 --rounds 3 --out gpurun_out/p8_tune.json > gpurun_out/p8_tune.txt 2>&1
