#!/bin/bash
# Round-2 (c) final: GPU suite, smoke(), default bench line (CPU baseline included), the rocprofv3
# kernel trace + stats of the bench command and its cross-check against the live event pairs.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf > gpurun_out/r2c_final_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r2c_final_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2c_smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/r2c_bench_final.json 2> gpurun_out/r2c_bench_final.err || exit $?
cat gpurun_out/r2c_bench_final.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2c_fkt -o kt -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r2c_fkt_bench.json 2> $R/gpurun_out/r2c_fkt.err || exit 1
cd $R && python3 scripts/rocprof_timed.py gpurun_out/r2c_fkt/kt_kernel_trace.csv gpurun_out/r2c_fkt_bench.json gpurun_out/r2c_final_rocprof_vs_bench.json
