#!/bin/bash
# Full GPU suite, the default bench line, the rocprofv3 kernel trace of the bench command, streams A/B.
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf > gpurun_out/r2b_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r2b_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/r2b_bench.json 2> gpurun_out/r2b_bench.err || exit $?
echo bench; cat gpurun_out/r2b_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r2b_kt -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r2b_kt_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/r2b_kt.err || exit $?
cd $GRAFT_REPO_ROOT
python3 scripts/rocprof_timed.py gpurun_out/r2b_kt/kt_kernel_trace.csv gpurun_out/r2b_kt_bench.json gpurun_out/r2b_kt_timed.json
for s in 1 2 4; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --streams $s > gpurun_out/r2b_streams$s.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r2b_streams$s.json')); print('streams $s', d['value'], d['ms_per_step'])"
done
