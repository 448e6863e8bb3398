#!/bin/bash
# broad single-layer sweep of the w6 bs8 1280 dispatch over every fragment / ring configuration
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5x; mkdir -p $O; cd $R
export PYTHONPATH=$R/yolo-series_amd:$R
C=17,201,204,231,232,239,262,270,271,272,273,274,275,276,277,280,281,282,283,284,285,286,287,288,290,291,292,293,294,295
timeout -k 10 900 python -u scripts/tune_ops.py --model yolov7-w6 --b 8 --img 1280 --cands $C --rounds 2 --out $O/tune_w6_all.json > $O/tune_w6_all.txt 2>&1 || { tail $O/tune_w6_all.txt; exit 1; }
grep -v amdgpu.ids $O/tune_w6_all.txt | awk '$10 > 1.5' | tail -40
tail -1 $O/tune_w6_all.txt
