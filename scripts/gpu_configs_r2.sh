#!/bin/bash
# Round-2 lines for the other BASELINE configs: [3] yolov7-w6 1280 bs8, [4] fp8, and tiny.
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD/yolo-series_amd:$PWD
timeout -k 10 400 python -u bench.py --model yolov7-w6 --img 1280 --batch 8 --steps 40 --no-cpu-baseline > gpurun_out/r2_bench_w6.json 2> gpurun_out/r2_bench_w6.err
timeout -k 10 300 python -u bench.py --dtype fp8 --steps 60 --no-cpu-baseline > gpurun_out/r2_bench_fp8b.json 2> gpurun_out/r2_bench_fp8b.err
timeout -k 10 300 python -u bench.py --steps 60 --no-cpu-baseline > gpurun_out/r2_bench_f16b.json 2> gpurun_out/r2_bench_f16b.err
timeout -k 10 300 python -u bench.py --model yolov7-tiny --steps 60 --no-cpu-baseline > gpurun_out/r2_bench_tiny.json 2> gpurun_out/r2_bench_tiny.err
