#!/bin/bash
# Round 3 (q): in-network single-layer sweep of the two ws64 forms (11 column-pair, 15 half-patch ring)
# on the 64-channel 3x3 layers (@320, @160 x4, @80 x3).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3q}
O=gpurun_out/$TAG
cd $R && mkdir -p $O
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 400 python -u scripts/tune_ops.py --ops 1,4,5,6,7,61,62,63 --cands 11,15 --rounds 3 > $O/tune.txt 2>&1 || { tail -20 $O/tune.txt; exit 1; }
grep -v amdgpu.ids $O/tune.txt
