#!/bin/bash
# Round 3 (m): persistent Detect head with the decode in the row pass — A/B vs the round-2 ring (99),
# then the GPU tests that cover the head.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3m}
cd $R && mkdir -p gpurun_out/$TAG
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 180 scripts/detbench 99,0,98,99,0 > gpurun_out/$TAG/det.txt 2>&1 || { cat gpurun_out/$TAG/det.txt; exit 1; }
cat gpurun_out/$TAG/det.txt
timeout -k 10 900 python -u -m pytest tests/test_variants.py tests/test_bench_config.py tests/test_gpu_forward.py tests/test_gpu_nms.py tests/test_detect.py tests/test_gpu_model_paths.py -m gpu -v -s --timeout 400 --timeout-method thread -rf > gpurun_out/$TAG/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/$TAG/tests.log | tail -2; grep -E "^FAILED" gpurun_out/$TAG/tests.log | head -20
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1; do
    YV7_DET_PRING=$v timeout -k 10 240 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/$TAG/bench_d${v}_$r.json 2> gpurun_out/$TAG/bench_d${v}_$r.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/$TAG/bench_d${v}_$r.json'));print('DET_PRING=$v round $r', d['value'], d['detail']['serial_forward_ms'])"
  done
done
