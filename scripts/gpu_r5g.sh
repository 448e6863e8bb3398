#!/bin/bash
# A/B of the division-free PixelWalk: test suite on the new library, convbench + PMC (instructions per
# MFMA, clock) of the 1x1 8-phase ring on new and base (libyv7_base.so) libraries.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5g; mkdir -p $O; cd $R
export PYTHONPATH=$R/yolo-series_amd:$R
L=$R/yolo-series_amd/yv7
cp $L/libyv7.so $L/libyv7_new.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
for lib in new base new base; do
  cp $L/libyv7_$lib.so $L/libyv7.so
  CB_SHAPE="1x1" timeout -k 10 200 ./scripts/convbench 0 > $O/cb_1x1_$lib.txt 2>&1 || exit 1
  tail -1 $O/cb_1x1_$lib.txt
done
for lib in new base; do
  cp $L/libyv7_$lib.so $L/libyv7.so
  bash scripts/pmc_cb.sh "1x1 1024->1024 @40" gpurun_out/r5g/pmc_$lib 0 > $O/pmc_$lib.txt 2>&1 || exit 1
  grep -A2 "p8_kernel" $O/pmc_$lib.txt
done
cp $L/libyv7_new.so $L/libyv7.so
