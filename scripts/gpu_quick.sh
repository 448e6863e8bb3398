#!/bin/bash
# Quick GPU iteration: gpu tests (optional filter $1) + per-op profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread ${1:+-k "$1"} > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python scripts/op_profile.py --iters 10 --top 0 --csv gpurun_out/ops.csv > gpurun_out/op_profile.txt 2>&1 || exit 1
cat gpurun_out/op_profile.txt
