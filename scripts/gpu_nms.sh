#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_nms.py tests/test_bench_config.py tests/test_integration.py tests/test_detect.py -v --timeout 300 --timeout-method thread -rf > gpurun_out/nms_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/nms_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/nms_kt -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/nms_kt_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/nms_kt.err || exit $?
cd $GRAFT_REPO_ROOT
grep -i "nms\|row_best" gpurun_out/nms_kt/kt_kernel_stats.csv | cut -c1-160
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/nms_bench.json 2>/dev/null || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/nms_bench.json')); print(d['value'], d['ms_per_step'], d['detail']['detect_py_split_ms'])"
