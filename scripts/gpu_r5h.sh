#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5h; mkdir -p $O; cd $R
for sh in "3x3s2 256->256" "3x3s2 512->512" "3x3s2 128->128 @80" "3x3s2 256->512" "3x3s2 512->768" "3x3s2 768->" "3x3s2 256->384" "3x3s2 384->"; do
  CB_SHAPE="$sh" timeout -k 10 120 ./scripts/convbench 0 274 277 278 279 231 232 >> $O/cb.txt 2>&1 || exit 1
done
grep -v total $O/cb.txt
