#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5o; mkdir -p $O; cd $R
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 500 python -u scripts/tune_ops.py --cands 290,291,292,293,294,295 --rounds 3 > $O/tune_v7.txt 2>&1 || { tail $O/tune_v7.txt; exit 1; }
grep -v amdgpu.ids $O/tune_v7.txt | awk '$NF != "" {print}' | grep -v "gain    0.0\|gain   -" | tail -40
timeout -k 10 500 python -u scripts/tune_ops.py --model yolov7-w6 --b 8 --img 1280 --cands 290,291,292,293,294,295 --rounds 3 > $O/tune_w6.txt 2>&1 || { tail $O/tune_w6.txt; exit 1; }
grep -v amdgpu.ids $O/tune_w6.txt | grep -v "gain    0.0\|gain   -" | tail -40
