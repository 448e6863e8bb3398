#!/bin/bash
# A/B of the wide-layer persistent-ring dispatch (YV7_WIDE_PRING=0 / default 1) on one box:
# GPU forward tests, per-op times, bench for yolov7 bs32 and yolov7-w6 bs8.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_forward.py tests/test_fp8.py -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/wide_tests.log 2>&1 && tail -1 gpurun_out/wide_tests.log &&
for w in 0 1 0 1; do
  YV7_WIDE_PRING=$w timeout -k 10 200 python scripts/op_profile.py --iters 10 --top 0 --csv gpurun_out/ops_wide$w.csv > gpurun_out/op_wide$w.txt 2>&1 || exit 1
  YV7_WIDE_PRING=$w timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b_wide$w.json 2>/dev/null || exit 1
  YV7_WIDE_PRING=$w timeout -k 10 200 python bench.py --no-cpu-baseline --model yolov7-w6 --img 1280 --batch 8 > gpurun_out/b_wide_w6_$w.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/b_wide$w.json'));e=json.load(open('gpurun_out/b_wide_w6_$w.json'));print('wide=$w p5',d['value'],d['detail']['forward_ms_events'],'w6',e['value'],e['detail']['forward_ms_events'])"
done
