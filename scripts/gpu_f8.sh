#!/bin/bash
# fp8: parity of the fused-quantization GEMM, then per-op A/B (fused vs staged vs fp16) and bench
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD/yolo-series_amd:$PWD
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp8.py > gpurun_out/f8_tests.log 2>&1
timeout -k 10 240 python -u scripts/ab_ops.py --fp8 0 --variants 0,81,82 --rounds 3 --out gpurun_out/f8_ab_all.json > gpurun_out/f8_ab_all.txt 2>&1
timeout -k 10 240 python -u scripts/ab_ops.py --fp8 512 --variants 0,81,82 --rounds 3 --out gpurun_out/f8_ab_prod.json > gpurun_out/f8_ab_prod.txt 2>&1
timeout -k 10 300 python -u bench.py --dtype fp8 --steps 40 --no-cpu-baseline > gpurun_out/f8_bench.json 2> gpurun_out/f8_bench.err
timeout -k 10 300 python -u bench.py --dtype fp8 --fp8-min-cout 0 --steps 40 --no-cpu-baseline > gpurun_out/f8_bench_all.json 2> gpurun_out/f8_bench_all.err
