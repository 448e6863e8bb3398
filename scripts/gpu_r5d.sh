#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5d; mkdir -p $O; cd $R
export PYTHONPATH=$R/yolo-series_amd:$R
CB_SHAPE="3x3s2 64->128" timeout -k 10 120 ./scripts/convbench 0 280 281 285 286 287 > $O/cb_s2.txt 2>&1 || exit 1
CB_SHAPE="3x3s2 128->" timeout -k 10 120 ./scripts/convbench 0 282 283 284 288 289 >> $O/cb_s2.txt 2>&1 || exit 1
cat $O/cb_s2.txt
timeout -k 10 600 python -u -m pytest tests/test_variants.py -m gpu -x -v --timeout 300 --timeout-method thread -rf -k "ragged or every_conv" > $O/tests.log 2>&1; tail -3 $O/tests.log
