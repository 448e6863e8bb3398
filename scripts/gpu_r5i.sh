#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5i; mkdir -p $O; cd $R
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 400 python -u scripts/tune_ops.py --ops 20,30,64,73 --cands 274,277,278,231,232 --rounds 3 > $O/tune_v7.txt 2>&1 || { tail $O/tune_v7.txt; exit 1; }
grep -v amdgpu.ids $O/tune_v7.txt | tail -5
timeout -k 10 400 python -u scripts/tune_ops.py --model yolov7-w6 --b 8 --img 1280 --ops 14,21,28,71,78,85 --cands 274,277,278,231,232 --rounds 3 > $O/tune_w6.txt 2>&1 || { tail $O/tune_w6.txt; exit 1; }
grep -v amdgpu.ids $O/tune_w6.txt | tail -7
