#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5y; mkdir -p $O; cd $R
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 400 python -u -m pytest tests/test_variants.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -1; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/tune_ops.py --model yolov7-w6 --b 8 --img 1280 --ops 6,64,67,68,69,23,24,25,26,30,33,42,87,88 --cands 302,303,293,204,17,276,273 --rounds 3 > $O/tune_w6.txt 2>&1 || { tail $O/tune_w6.txt; exit 1; }
grep -v amdgpu.ids $O/tune_w6.txt | tail -15
timeout -k 10 400 python -u scripts/tune_ops.py --ops 54,58,59,60,32,33,34,35,38,44 --cands 302,303,17,276,273 --rounds 3 > $O/tune_v7.txt 2>&1 || { tail $O/tune_v7.txt; exit 1; }
grep -v amdgpu.ids $O/tune_v7.txt | tail -11
