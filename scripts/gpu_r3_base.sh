#!/bin/bash
# Round 3 baseline on this round's box: GPU suite, default bench line, serial per-op profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r3
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf > gpurun_out/r3/base_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r3/base_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r3/base_bench.json 2> gpurun_out/r3/base_bench.err || exit $?
cat gpurun_out/r3/base_bench.json
timeout -k 10 300 python -u scripts/op_profile.py --top 90 > gpurun_out/r3/base_ops.txt 2>&1 || exit $?
head -5 gpurun_out/r3/base_ops.txt
