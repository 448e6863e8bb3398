#!/bin/bash
# After a kernel change: the variant / bench-config / forward parity tests, a per-op profile and two
# default bench runs.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 600 python -u -m pytest tests/test_variants.py tests/test_bench_config.py tests/test_gpu_forward.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/cp_tests.log 2>&1 || { tail -40 gpurun_out/cp_tests.log; exit 1; }
tail -2 gpurun_out/cp_tests.log
timeout -k 10 200 python -u scripts/op_profile.py --top 30 > gpurun_out/cp_ops.txt 2>&1 || { tail gpurun_out/cp_ops.txt; exit 1; }
grep -A40 "^forward" gpurun_out/cp_ops.txt | head -42
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/cp_b$i.json 2> gpurun_out/cp_b$i.err || { tail gpurun_out/cp_b$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['detail']['serial_forward_ms'])" gpurun_out/cp_b$i.json
done
