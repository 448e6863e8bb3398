#!/bin/bash
# Round 3 (u): candidate sweep on the big 1x1 / stride-2 layers of the current graph.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3u}
O=gpurun_out/$TAG
cd $R && mkdir -p $O
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 900 python -u scripts/tune_ops.py --ops 17,19,2,11,26,29,56,12 --cands 201,202,203,204,205,206,211,212,213,214,215,216,217,231,232 --rounds 2 > $O/tune.txt 2>&1 || { tail -20 $O/tune.txt; exit 1; }
grep -v amdgpu.ids $O/tune.txt
