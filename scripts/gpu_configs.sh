#!/bin/bash
# Bench lines of the non-headline configs (fp8 1x1 convs; yolov7-w6 1280 bs8) at the bench defaults.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --dtype fp8 --no-cpu-baseline > gpurun_out/bench_fp8.json 2> gpurun_out/bench_fp8.err &&
timeout -k 10 300 python bench.py --model yolov7-w6 --img 1280 --batch 8 --no-cpu-baseline > gpurun_out/bench_w6.json 2> gpurun_out/bench_w6.err &&
timeout -k 10 300 python bench.py --model yolov7-w6 --img 1280 --batch 8 --no-cpu-baseline --streams 2 > gpurun_out/bench_w6_s2.json 2>> gpurun_out/bench_w6.err &&
for f in bench_fp8 bench_w6 bench_w6_s2; do python -c "import json;d=json.load(open('gpurun_out/$f.json'));print('$f',d['value'],d['ms_per_step'],d['detail']['streams'])"; done
