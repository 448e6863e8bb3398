#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5w8; mkdir -p $O; cd $R
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 400 python -u -m pytest tests/test_variants.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -1; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/tune_ops.py --ops 17,19,21,48,65,61 --cands 295,304,292 --rounds 3 > $O/tune_v7.txt 2>&1 || { tail $O/tune_v7.txt; exit 1; }
grep -v amdgpu.ids $O/tune_v7.txt | tail -7 | cut -c1-190
timeout -k 10 400 python -u scripts/tune_ops.py --model yolov7-w6 --b 8 --img 1280 --ops 13,15,56,72,70 --cands 295,304,292 --rounds 3 > $O/tune_w6.txt 2>&1 || { tail $O/tune_w6.txt; exit 1; }
grep -v amdgpu.ids $O/tune_w6.txt | tail -6 | cut -c1-190
