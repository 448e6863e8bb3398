#!/bin/bash
# Config bench lines at the defaults + a streams 2/3/4 re-check (same box).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --dtype fp8 --no-cpu-baseline > gpurun_out/bench_fp8.json 2> gpurun_out/bench_fp8.err &&
python -c "import json;d=json.load(open('gpurun_out/bench_fp8.json'));print('fp8',d['value'],d['ms_per_step'])" &&
STREAMS="3 2 4 3" bash scripts/ab_streams.sh
