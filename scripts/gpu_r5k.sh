#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5k; mkdir -p $O; cd $R
export PYTHONPATH=$R/yolo-series_amd:$R
CB_SHAPE="1x1" timeout -k 10 200 ./scripts/convbench 0 290 291 292 293 294 295 > $O/cb_1x1.txt 2>&1 || { cat $O/cb_1x1.txt; exit 1; }
cat $O/cb_1x1.txt
timeout -k 10 600 python -u -m pytest tests/test_variants.py -m gpu -x -v --timeout 300 --timeout-method thread -rf -k "ragged or every_conv" > $O/tests.log 2>&1; tail -3 $O/tests.log
