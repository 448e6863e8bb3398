#!/bin/bash
# Round 2 (c): GPU suite, default bench line, and a rocprofv3 kernel trace of the bench command to
# check the live per-op event pairs (hipExtLaunchKernel) against the trace's kernel durations.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2c_tests.log 2>&1 || { tail -40 gpurun_out/r2c_tests.log; exit 1; }
tail -2 gpurun_out/r2c_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r2c_bench.json 2> gpurun_out/r2c_bench.err || { tail gpurun_out/r2c_bench.err; exit 1; }
cat gpurun_out/r2c_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2c_kt -o kt -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r2c_kt_bench.json 2> $R/gpurun_out/r2c_kt.err || exit 1
cd $R && python3 scripts/rocprof_timed.py gpurun_out/r2c_kt/kt_kernel_trace.csv gpurun_out/r2c_kt_bench.json gpurun_out/r2c_rocprof_vs_bench.json
