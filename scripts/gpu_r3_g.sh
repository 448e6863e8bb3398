#!/bin/bash
# Round 3 (g): hring dummy-DMA fix — microbenchmark of the two halo-ring shapes, then the full (f) pass.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3c}
cd $R && mkdir -p gpurun_out/$TAG
CB_SHAPE="3x3 128->128 @80" timeout -k 10 120 scripts/convbench 0 262 913 262 > gpurun_out/$TAG/hooks.txt 2>&1 || { cat gpurun_out/$TAG/hooks.txt; exit 1; }
CB_SHAPE="3x3 128->256 @80" timeout -k 10 120 scripts/convbench 0 262 >> gpurun_out/$TAG/hooks.txt 2>&1 || exit 1
cat gpurun_out/$TAG/hooks.txt
bash scripts/gpu_r3_f.sh $TAG
