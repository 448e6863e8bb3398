#!/bin/bash
# Round 3 (aa): GPU suite, then the Detect-head epilogue order A/B (YV7_DET_PIPE 0 / 1 / 2) in-network.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3aa}
O=gpurun_out/$TAG
cd $R && mkdir -p $O
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -2; grep -E "^FAILED" $O/tests.log | head
[ $rc -eq 0 ] || exit $rc
for rep in a b; do
for m in 0 1 2; do
  YV7_DET_PIPE=$m timeout -k 10 300 python -u scripts/op_profile.py --top 100 > $O/ops_${m}$rep.txt 2>&1 || exit 1
  echo "pipe=$m$rep $(head -2 $O/ops_${m}$rep.txt | tail -1)"; grep -E "^ *8[345] DET" $O/ops_${m}$rep.txt
done
done
