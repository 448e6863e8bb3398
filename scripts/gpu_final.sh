#!/bin/bash
# End-of-round evidence on the current tree: GPU suite + smoke, then scripts/gpu_prof.sh
# (serial kernel trace, PMC traffic, bench line, bench kernel trace, roofline cross-check).
# usage: bash scripts/gpu_final.sh TAG TREE
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r4}; TREE=${2:-}
O=gpurun_out/$TAG
cd $R && mkdir -p $O
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/gpu_tests.log | tail -2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash scripts/gpu_prof.sh $TAG $TREE
