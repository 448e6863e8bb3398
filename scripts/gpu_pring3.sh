#!/bin/bash
# Variant 218 (128x128 persistent ring, BK 32 x 3 stages, three blocks per CU): correctness on every
# conv of yolov7 / tiny, single-layer sweep vs the dispatch, bench A/B (YV7_PRING3).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 200 python -u scripts/check_variant.py 218 > gpurun_out/p3_check.log 2>&1 || { tail -20 gpurun_out/p3_check.log; exit 1; }
timeout -k 10 200 python -u scripts/check_variant.py 218 yolov7-tiny 2 192 256 >> gpurun_out/p3_check.log 2>&1 || { tail -20 gpurun_out/p3_check.log; exit 1; }
grep variant gpurun_out/p3_check.log
timeout -k 10 400 python -u scripts/tune_ops.py --cands 0,218,204 > gpurun_out/p3_tune.txt 2>&1 || { tail -20 gpurun_out/p3_tune.txt; exit 1; }
grep -E "best +218|sum of" gpurun_out/p3_tune.txt
bash scripts/gpu_ab_env.sh p3 YV7_PRING3 0 1 2
