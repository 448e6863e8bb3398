#!/bin/bash
# exact fast path of the row-score scan: detbench, the head's parity tests, in-network ops
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5rs; mkdir -p $O; cd $R
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 120 ./scripts/detbench 0,94,0,94 > $O/detbench.txt 2>&1 || { cat $O/detbench.txt; exit 1; }
cat $O/detbench.txt
timeout -k 10 600 python -u -m pytest tests/test_bench_config.py tests/test_gpu_nms.py tests/test_variants.py tests/test_detect.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -1; grep -E "^FAILED|Error" $O/tests.log | head -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/op_profile.py --top 100 > $O/ops.txt 2>&1 || exit 1
grep -E "^forward| DET" $O/ops.txt | head -4
