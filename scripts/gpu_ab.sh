#!/bin/bash
# Parity of the new kernel configurations / NMS path first, then the per-op A/B and a bench line
# (only if parity is green).
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_variants.py tests/test_bench_config.py tests/test_gpu_model_paths.py tests/test_gpu_nms.py tests/test_integration.py -v --timeout 300 --timeout-method thread -rf > gpurun_out/ab_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -8 gpurun_out/ab_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/ab_ops.py --variants ${VARIANTS:-0,221,222,223,201,204} --out gpurun_out/ab_ops.json > gpurun_out/ab_ops.txt 2>&1
rc=$?
echo "ab rc=$rc"; tail -12 gpurun_out/ab_ops.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab_bench.json 2> gpurun_out/ab_bench.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/ab_bench.json
exit $rc
