#!/bin/bash
# Round-2 GPU check: the GPU test suite, then the default bench line.  A test failure (rc 1) still
# lets the bench run; a fault / abort / timeout (any other rc) ends the call.
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf ${PYTEST_ARGS} > gpurun_out/r2_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/r2_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > gpurun_out/r2_bench.json 2> gpurun_out/r2_bench.err
brc=$?
echo "bench rc=$brc"
cat gpurun_out/r2_bench.json
exit $brc
