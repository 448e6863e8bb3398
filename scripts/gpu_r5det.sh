#!/bin/bash
# pipelined Detect head: microbenchmark vs the round-3 form (94), then the head's parity tests
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5det2; mkdir -p $O; cd $R
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 120 ./scripts/detbench 0,94,0,94 > $O/detbench.txt 2>&1 || { cat $O/detbench.txt; exit 1; }
cat $O/detbench.txt
timeout -k 10 600 python -u -m pytest tests/test_bench_config.py tests/test_gpu_nms.py tests/test_variants.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -2; grep -E "^FAILED|Error" $O/tests.log | head -5; exit $rc
