#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5r; mkdir -p $O; cd $R
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 400 python -u scripts/tune_ops.py --ops 1,4,5,13,14,57,58,80 --cands 285,286,287,288 --rounds 3 > $O/tune_v7.txt 2>&1 || { tail $O/tune_v7.txt; exit 1; }
grep -v amdgpu.ids $O/tune_v7.txt | tail -9
timeout -k 10 400 python -u scripts/tune_ops.py --model yolov7-w6 --b 8 --img 1280 --ops 2,3,9,10,66,92 --cands 285,286,287,288 --rounds 3 > $O/tune_w6.txt 2>&1 || { tail $O/tune_w6.txt; exit 1; }
grep -v amdgpu.ids $O/tune_w6.txt | tail -7
