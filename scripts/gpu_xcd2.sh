#!/bin/bash
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD/yolo-series_amd:$PWD
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bench_config.py tests/test_variants.py > gpurun_out/xcd2_tests.log 2>&1
timeout -k 10 300 python -u scripts/op_profile.py --iters 4 --top 30 > gpurun_out/xcd2_ops.txt 2>&1
bash scripts/pmc_traffic.sh
python3 scripts/pmc_traffic.py gpurun_out gpurun_out/xcd2_pmc_traffic.json
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 60 --no-cpu-baseline > gpurun_out/xcd2_bench_$i.json 2> gpurun_out/xcd2_bench_$i.err
done
