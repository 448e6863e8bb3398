#!/bin/bash
# Round 3 (k): halo ring, compact (262) vs spread (915) epilogue placement; two interleaved rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3k}
cd $R && mkdir -p gpurun_out/$TAG
for shp in "3x3 128->128 @80" "3x3 128->256 @80"; do
  CB_SHAPE="$shp" timeout -k 10 120 scripts/convbench 262 915 913 262 915 >> gpurun_out/$TAG/spread.txt 2>&1 || { cat gpurun_out/$TAG/spread.txt; exit 1; }
done
cat gpurun_out/$TAG/spread.txt
