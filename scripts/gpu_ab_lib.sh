#!/bin/bash
# A/B of two builds of libyv7 (abtmp/libyv7_base.so vs abtmp/libyv7_new.so) in one box: interleaved
# default bench runs, a per-op profile of each, then the parity tests on the new build.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export PYTHONPATH=$R/yolo-series_amd:$R
L=yolo-series_amd/yv7/libyv7.so
for v in base new; do
  cp abtmp/libyv7_$v.so $L
  timeout -k 10 200 python -u scripts/op_profile.py --top 0 > gpurun_out/abl_ops_$v.txt 2>&1 || { tail gpurun_out/abl_ops_$v.txt; exit 1; }
  grep -A9 "^CONV k3s1" gpurun_out/abl_ops_$v.txt | sed "s/^/$v /"; grep "^forward" gpurun_out/abl_ops_$v.txt
done
for i in 1 2; do for v in base new; do
  cp abtmp/libyv7_$v.so $L
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/abl_${v}_$i.json 2> gpurun_out/abl_${v}_$i.err || { tail gpurun_out/abl_${v}_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['detail']['serial_forward_ms'])" gpurun_out/abl_${v}_$i.json
done; done
cp abtmp/libyv7_new.so $L
timeout -k 10 600 python -u -m pytest tests/test_variants.py tests/test_bench_config.py tests/test_gpu_forward.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abl_tests.log 2>&1 || { tail -30 gpurun_out/abl_tests.log; exit 1; }
tail -2 gpurun_out/abl_tests.log
