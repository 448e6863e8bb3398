#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5q; mkdir -p $O; cd $R
export PYTHONPATH=$R/yolo-series_amd:$R
for sh in "3x3 64->" "3x3 128->" "3x3s2 64->" "3x3s2 128->128"; do
  CB_SHAPE="$sh" timeout -k 10 150 ./scripts/convbench 0 280 282 283 285 286 287 288 >> $O/cb.txt 2>&1 || { cat $O/cb.txt; exit 1; }
done
grep -v total $O/cb.txt
timeout -k 10 600 python -u -m pytest tests/test_variants.py -m gpu -x -v --timeout 300 --timeout-method thread -rf -k "ragged or every_conv or rejects" > $O/tests.log 2>&1; tail -3 $O/tests.log
