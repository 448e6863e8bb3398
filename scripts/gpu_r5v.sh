#!/bin/bash
# cin-1024 register-weight 1x1 rows (302-305): variant tests, then one layer forced at a time
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5v; mkdir -p $O; cd $R
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 400 python -u -m pytest tests/test_variants.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -1; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/tune_ops.py --ops 26,29,36,37,74,53,70,28,31,45 --cands 302,303,304,305 --rounds 3 > $O/tune_v7.txt 2>&1 || { tail $O/tune_v7.txt; exit 1; }
grep -v amdgpu.ids $O/tune_v7.txt | tail -11
