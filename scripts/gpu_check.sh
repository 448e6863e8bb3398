#!/bin/bash
# Dispatch change check: GPU forward tests, per-op times, bench (yolov7 bs32, yolov7-w6 bs8).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_forward.py -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/chk_tests.log 2>&1 && tail -1 gpurun_out/chk_tests.log &&
timeout -k 10 200 python scripts/op_profile.py --iters 10 --top 0 --csv gpurun_out/ops_chk.csv > gpurun_out/op_chk.txt 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b_chk.json 2>/dev/null &&
timeout -k 10 200 python bench.py --no-cpu-baseline --model yolov7-w6 --img 1280 --batch 8 > gpurun_out/b_chk_w6.json 2>/dev/null &&
python -c "import json;d=json.load(open('gpurun_out/b_chk.json'));e=json.load(open('gpurun_out/b_chk_w6.json'));print('p5',d['value'],d['detail']['forward_ms_events'],'w6',e['value'],e['detail']['forward_ms_events'])"
