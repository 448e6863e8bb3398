#!/bin/bash
# yolov7-w6 1280 bs8: GPU forward tests, per-op profile, bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_forward.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/w6_tests.log 2>&1 && tail -2 gpurun_out/w6_tests.log &&
timeout -k 10 200 python scripts/op_profile.py --model yolov7-w6 --img 1280 --b 8 --iters 10 --top 0 --csv gpurun_out/ops_w6b.csv > gpurun_out/op_w6b.txt 2>&1 &&
timeout -k 10 300 python bench.py --model yolov7-w6 --img 1280 --batch 8 --no-cpu-baseline > gpurun_out/bench_w6.json 2> gpurun_out/bench_w6.err &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_p5.json 2> gpurun_out/bench_p5.err &&
for f in bench_w6 bench_p5; do python -c "import json;d=json.load(open('gpurun_out/$f.json'));print('$f',d['value'],d['ms_per_step'])"; done
