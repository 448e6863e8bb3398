#!/bin/bash
# Round 3 (y): every conv op of the current yolov7 bs32 graph with each candidate configuration forced
# on it alone (the rest on the dispatch), 2 interleaved rounds: where the dispatch is no longer the best.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3y}
O=gpurun_out/$TAG
cd $R && mkdir -p $O
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 1100 python -u scripts/tune_ops.py --cands 201,202,203,204,205,206,217,231,232,239,262,11,15,4,5,6,7,8,110,112,120,122,130,132,140 --rounds 2 --iters 2 --out $O/tune.json > $O/tune.txt 2>&1 || { tail -20 $O/tune.txt; exit 1; }
grep -v amdgpu.ids $O/tune.txt | tail -90
