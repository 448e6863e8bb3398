#!/bin/bash
# Round 3 (n): the whole GPU suite + smoke on the current tree, then the profile pipeline (serial kernel
# trace, per-kernel PMC traffic, bench line, bench kernel trace, roofline cross-check).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3n}
cd $R && mkdir -p gpurun_out/$TAG
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf > gpurun_out/$TAG/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/$TAG/tests.log | tail -2; grep -E "^FAILED" gpurun_out/$TAG/tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { cat gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
bash scripts/gpu_r3_prof.sh $TAG "${2:-}"
