#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3t}
O=gpurun_out/$TAG
cd $R && mkdir -p $O
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 200 python -u scripts/diag_pool.py 9 > $O/pool9.txt 2>&1; echo "rc=$?"; grep -v amdgpu.ids $O/pool9.txt | tail -20
