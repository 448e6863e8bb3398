#!/bin/bash
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD/yolo-series_amd:$PWD
for i in 1 2; do
  for s in 2 3 4; do
    timeout -k 10 300 python -u bench.py --steps 60 --no-cpu-baseline --streams $s > gpurun_out/st_${s}_$i.json 2> gpurun_out/st_${s}_$i.err
  done
done
