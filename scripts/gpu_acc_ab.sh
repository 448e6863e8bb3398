#!/bin/bash
# Accuracy A/B of two builds against the fp32 oracle at the bench configuration (bs 32, 640):
# tests/test_bench_config.py's per-layer rms-rel and z errors, printed for each build.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export PYTHONPATH=$R/yolo-series_amd:$R
L=yolo-series_amd/yv7/libyv7.so
for v in base new; do
  cp abtmp/libyv7_$v.so $L
  timeout -k 10 400 python -u -m pytest tests/test_bench_config.py -m gpu -s -q --timeout 300 --timeout-method thread > gpurun_out/acc_$v.log 2>&1 || { tail -20 gpurun_out/acc_$v.log; exit 1; }
  grep -E "oracle images|z vs fp32|bs32 fp16:" gpurun_out/acc_$v.log | sed "s/^/$v: /" | cut -c1-300
done
cp abtmp/libyv7_new.so $L
