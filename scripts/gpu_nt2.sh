#!/bin/bash
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD/yolo-series_amd:$PWD
for nt in 1 0; do
  YV7_STORE_NT=$nt timeout -k 10 300 python -u scripts/op_profile.py --iters 4 --top 14 > gpurun_out/nt2_ops_$nt.txt 2>&1
done
for i in 1 2; do
  for nt in 1 0; do
    YV7_STORE_NT=$nt timeout -k 10 300 python -u bench.py --steps 60 --no-cpu-baseline > gpurun_out/nt2_bench_${nt}_$i.json 2> gpurun_out/nt2_bench_${nt}_$i.err
  done
done
