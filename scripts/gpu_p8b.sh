#!/bin/bash
# full GPU suite on the new dispatch, then bench A/B of the 8-phase ring (interleaved processes)
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD/yolo-series_amd:$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/p8b_tests.log 2>&1
for i in 1 2; do
  YV7_P8=1 timeout -k 10 300 python -u bench.py --steps 60 --no-cpu-baseline > gpurun_out/p8b_bench_on_$i.json 2> gpurun_out/p8b_bench_on_$i.err
  YV7_P8=0 timeout -k 10 300 python -u bench.py --steps 60 --no-cpu-baseline > gpurun_out/p8b_bench_off_$i.json 2> gpurun_out/p8b_bench_off_$i.err
done
