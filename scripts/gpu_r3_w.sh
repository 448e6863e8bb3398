#!/bin/bash
# Round 3 (w): N-split weight-stationary 1x1 ring (variant 239): forced-variant parity on every layer
# shape, then single-layer timing on the short-K 256-channel 1x1 layers.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3w}
O=gpurun_out/$TAG
cd $R && mkdir -p $O
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 300 python -u -m pytest tests/test_variants.py -m gpu -x -v --timeout 240 --timeout-method thread -rf > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -2; grep -E "^FAILED|Error" $O/tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/tune_ops.py --ops 8,12,56,17 --cands 239,234,231 --rounds 3 > $O/tune.txt 2>&1 || { tail -20 $O/tune.txt; exit 1; }
grep -v amdgpu.ids $O/tune.txt
