#!/bin/bash
# fp8 config (BASELINE configs[4]): GPU fp8 tests, bench line, per-op profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fp8.py -x -v -s -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/fp8_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --dtype fp8 --no-cpu-baseline > gpurun_out/bench_fp8.json 2> gpurun_out/bench_fp8.err &&
timeout -k 10 200 python scripts/op_profile.py --dtype fp8 --iters 10 --top 0 --csv gpurun_out/ops_fp8.csv > gpurun_out/op_profile_fp8.txt 2>&1 &&
cat gpurun_out/bench_fp8.json && tail -3 gpurun_out/fp8_tests.log
