#!/bin/bash
# Round 3 (f): the tree with the halo ring in the dispatch — GPU suite, smoke(), then the per-kernel
# profiling pipeline + default bench line (scripts/gpu_r3_prof.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3b}
cd $R && mkdir -p gpurun_out/$TAG
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread -rf > gpurun_out/$TAG/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/$TAG/tests.log | tail -2; grep -E "^FAILED" gpurun_out/$TAG/tests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG/smoke.log
bash scripts/gpu_r3_prof.sh $TAG "$(cat TREE_ID 2>/dev/null)"
