#!/bin/bash
# Round-2 final: the GPU test suite, smoke(), and the default bench line (CPU baseline included).
mkdir -p gpurun_out
export PYTHONPATH=$PWD/yolo-series_amd:$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf > gpurun_out/r2_final_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r2_final_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/r2_bench_final.json 2> gpurun_out/r2_bench_final.err || exit $?
cat gpurun_out/r2_bench_final.json
