#!/bin/bash
# Round 3 (j): Detect head epilogue breakdown (hooks 94 no K loop, 95 + no staging, 96 + temporal stores).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3j}
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 180 scripts/detbench 0,90,94,95,96,93,0 > gpurun_out/$TAG/det_hooks.txt 2>&1 || { cat gpurun_out/$TAG/det_hooks.txt; exit 1; }
cat gpurun_out/$TAG/det_hooks.txt
