#!/bin/bash
# broad single-layer sweep of the yolov7 bs32 640 dispatch over every fragment / ring configuration
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5aa; mkdir -p $O; cd $R
export PYTHONPATH=$R/yolo-series_amd:$R
C=17,204,231,232,262,270,271,272,273,274,275,276,277,278,279,280,281,282,283,284,285,286,287,288,290,291,292,293,294,295,302,303
timeout -k 10 1000 python -u scripts/tune_ops.py --cands $C --rounds 2 --out $O/tune_v7_all.json > $O/tune_v7_all.txt 2>&1 || { tail $O/tune_v7_all.txt; exit 1; }
grep -v amdgpu.ids $O/tune_v7_all.txt | awk '{for(i=1;i<=NF;i++) if($i=="gain" && $(i+1) > 1.5) print}' | cut -c1-200
tail -1 $O/tune_v7_all.txt
