#!/bin/bash
# register-weight Detect head: microbenchmark (0 = new default, 94 = staged-weight head), K = 512 form via
# YV7_DET_RW=2, then the parity tests that cover the head
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5rw; mkdir -p $O; cd $R
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 120 ./scripts/detbench 0,94,0,94 > $O/detbench.txt 2>&1 || { cat $O/detbench.txt; exit 1; }
cat $O/detbench.txt
YV7_DET_RW=2 timeout -k 10 120 ./scripts/detbench 0,94 > $O/detbench_rw2.txt 2>&1 || { cat $O/detbench_rw2.txt; exit 1; }
cat $O/detbench_rw2.txt
timeout -k 10 600 python -u -m pytest tests/test_bench_config.py tests/test_gpu_nms.py tests/test_variants.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -2; grep -E "^FAILED|Error" $O/tests.log | head -5; exit $rc
