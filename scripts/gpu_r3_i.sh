#!/bin/bash
# Round 3 (i): where the 64-channel 3x3 kernel (ws64) and the Detect head spend their time (hooks).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3i}
cd $R && mkdir -p gpurun_out/$TAG
CB_SHAPE="3x3 64->64 @" timeout -k 10 180 scripts/convbench 0 12 13 14 16 0 > gpurun_out/$TAG/ws64_hooks.txt 2>&1 || { cat gpurun_out/$TAG/ws64_hooks.txt; exit 1; }
cat gpurun_out/$TAG/ws64_hooks.txt
timeout -k 10 180 scripts/detbench 0,90,93,94,92,97,0 > gpurun_out/$TAG/det_hooks.txt 2>&1 || { cat gpurun_out/$TAG/det_hooks.txt; exit 1; }
cat gpurun_out/$TAG/det_hooks.txt
