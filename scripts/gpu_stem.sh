#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_bench_config.py tests/test_gpu_forward.py tests/test_detect.py tests/test_variants.py -v --timeout 300 --timeout-method thread -rf -k "not variant_api" > gpurun_out/stem_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/stem_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u scripts/op_profile.py --iters 10 --top 12 > gpurun_out/stem_ops.txt 2>&1
rc=$?; echo "prof rc=$rc"; head -16 gpurun_out/stem_ops.txt
YV7_STEM_OCC=3 timeout -k 10 200 python -u scripts/op_profile.py --iters 10 --top 3 > gpurun_out/stem_ops3.txt 2>&1
head -5 gpurun_out/stem_ops3.txt
