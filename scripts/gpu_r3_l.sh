#!/bin/bash
# Round 3 (l): halo-ring spread epilogue A/B, persistent Detect head A/B, then the GPU tests that
# cover both (variants, bench-config op checks, forward parity, NMS end to end).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3l}
cd $R && mkdir -p gpurun_out/$TAG
export PYTHONPATH=$R/yolo-series_amd:$R
for shp in "3x3 128->128 @80" "3x3 128->256 @80"; do
  CB_SHAPE="$shp" timeout -k 10 120 scripts/convbench 262 915 913 262 915 >> gpurun_out/$TAG/spread.txt 2>&1 || { cat gpurun_out/$TAG/spread.txt; exit 1; }
done
cat gpurun_out/$TAG/spread.txt
timeout -k 10 180 scripts/detbench 99,0,98,90,99,0 > gpurun_out/$TAG/det.txt 2>&1 || { cat gpurun_out/$TAG/det.txt; exit 1; }
cat gpurun_out/$TAG/det.txt
timeout -k 10 900 python -u -m pytest tests/test_variants.py tests/test_bench_config.py tests/test_gpu_forward.py tests/test_gpu_nms.py tests/test_detect.py -m gpu -v -s --timeout 400 --timeout-method thread -rf > gpurun_out/$TAG/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/$TAG/tests.log | tail -2; grep -E "^FAILED" gpurun_out/$TAG/tests.log | head -20
exit $rc
