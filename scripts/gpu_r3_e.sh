#!/bin/bash
# Round 3 (e): the halo ring with its epilogue pipelined into the next tile (variant 262).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r3
export PYTHONPATH=$R/yolo-series_amd:$R
CB_SHAPE="3x3 128->128 @80" timeout -k 10 120 scripts/convbench 0 262 913 262 > gpurun_out/r3/e_hooks.txt 2>&1 || { cat gpurun_out/r3/e_hooks.txt; exit 1; }
CB_SHAPE="3x3 128->256 @80" timeout -k 10 120 scripts/convbench 0 262 >> gpurun_out/r3/e_hooks.txt 2>&1 || exit 1
cat gpurun_out/r3/e_hooks.txt
for shp in "2 256 256" "2 640 640"; do
  timeout -k 10 240 python -u scripts/check_variant.py 262 yolov7 $shp >> gpurun_out/r3/e_check.log 2>&1 || { echo "check 262 $shp failed"; tail -20 gpurun_out/r3/e_check.log; exit 1; }
done
grep variant gpurun_out/r3/e_check.log
