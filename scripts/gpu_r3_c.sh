#!/bin/bash
# Round 3 (c): the column-group halo ring (variant 262): parity on every applicable layer, single-layer
# timing sweep vs 260 and the dispatch, PMC passes; then the new SPP cascade / variants through the suite.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r3
export PYTHONPATH=$R/yolo-series_amd:$R
for shp in "2 256 256" "2 640 640"; do
  timeout -k 10 240 python -u scripts/check_variant.py 262 yolov7 $shp >> gpurun_out/r3/c_check.log 2>&1 || { echo "check 262 $shp failed"; tail -20 gpurun_out/r3/c_check.log; exit 1; }
done
grep variant gpurun_out/r3/c_check.log
timeout -k 10 300 python -u scripts/tune_ops.py --ops 13,14,15,16,83 --cands 260,262 --rounds 3 > gpurun_out/r3/c_tune.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r3/c_tune.txt
bash scripts/pmc_cb.sh "3x3 128->128 @80" gpurun_out/r3/pmc_262 262 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_variants.py tests/test_bench_config.py tests/test_bench_contract.py -m gpu -v --timeout 300 --timeout-method thread -rf > gpurun_out/r3/c_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r3/c_tests.log | tail -2; grep -E "^FAILED" gpurun_out/r3/c_tests.log | head
