#!/bin/bash
# A/B of the split-K-in-four tile threshold (YV7_SPLIT4_TILES) on yolov7 640 bs32: per-op times + bench.
set -o pipefail
mkdir -p gpurun_out
for t in 128 256 400; do
  YV7_SPLIT4_TILES=$t timeout -k 10 200 python scripts/op_profile.py --iters 10 --top 0 --csv gpurun_out/ops_s4_$t.csv > gpurun_out/op_s4_$t.txt 2>&1 || exit 1
  YV7_SPLIT4_TILES=$t timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b_s4_$t.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/b_s4_$t.json'));print('split4 tiles<=$t',d['value'],d['ms_per_step'])"
done
