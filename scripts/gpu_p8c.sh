#!/bin/bash
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD/yolo-series_amd:$PWD
timeout -k 10 120 python -u scripts/check_variant.py 232 yolov7 2 256 256 > gpurun_out/p8c_check.log 2>&1
timeout -k 10 120 python -u scripts/check_variant.py 232 yolov7 4 640 640 >> gpurun_out/p8c_check.log 2>&1
timeout -k 10 120 python -u scripts/check_variant.py 232 yolov7-tiny 3 320 448 >> gpurun_out/p8c_check.log 2>&1
timeout -k 10 600 python -u scripts/tune_ops.py --cands 232,231 --rounds 3 --ops 2,3,8,10,11,12,13,14,19,20,22,30,32,38,43,51,52,58,59,60,64,66,67,76,78,83 --out gpurun_out/p8c_tune.json > gpurun_out/p8c_tune.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/p8b_tests.log 2>&1
for i in 1 2; do
  YV7_P8=1 timeout -k 10 300 python -u bench.py --steps 60 --no-cpu-baseline > gpurun_out/p8b_bench_on_$i.json 2> gpurun_out/p8b_bench_on_$i.err
  YV7_P8=0 timeout -k 10 300 python -u bench.py --steps 60 --no-cpu-baseline > gpurun_out/p8b_bench_off_$i.json 2> gpurun_out/p8b_bench_off_$i.err
done
