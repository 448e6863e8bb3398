#!/bin/bash
# fp8 config: which 1x1 convs go e4m3 (bench --fp8-min-cout) at the default 3 batches in flight.
set -o pipefail
mkdir -p gpurun_out
for c in 512 1024 256 0 512; do
  timeout -k 10 300 python bench.py --dtype fp8 --no-cpu-baseline --fp8-min-cout $c > gpurun_out/b_fp8_$c.json 2> gpurun_out/b_fp8.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/b_fp8_$c.json'));print('fp8 min_cout $c',d['value'],d['ms_per_step'])"
done
