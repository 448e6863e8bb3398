#!/bin/bash
# Round 3 (d): cost breakdown of the column-group halo ring (convbench hooks 911-914), then the
# per-kernel profiling pipeline on the current tree (scripts/gpu_r3_prof.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r3
export PYTHONPATH=$R/yolo-series_amd:$R
CB_SHAPE="3x3 128->128 @80" timeout -k 10 120 scripts/convbench 0 262 911 912 913 914 262 > gpurun_out/r3/d_hooks.txt 2>&1 || { cat gpurun_out/r3/d_hooks.txt; exit 1; }
CB_SHAPE="3x3 128->256 @80" timeout -k 10 120 scripts/convbench 0 262 914 >> gpurun_out/r3/d_hooks.txt 2>&1 || exit 1
cat gpurun_out/r3/d_hooks.txt
bash scripts/gpu_r3_prof.sh r3 "$(cat TREE_ID 2>/dev/null)"
