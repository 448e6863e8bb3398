#!/bin/bash
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD/yolo-series_amd:$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bench_config.py tests/test_variants.py > gpurun_out/ws2_tests.log 2>&1
for i in 1 2; do
  for w in 1 0; do
    YV7_WS1=$w timeout -k 10 300 python -u bench.py --steps 60 --no-cpu-baseline > gpurun_out/ws2_bench_${w}_$i.json 2> gpurun_out/ws2_bench_${w}_$i.err
  done
done
