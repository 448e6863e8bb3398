#!/bin/bash
# A/B: batches in flight (bench --streams) vs the single-stream pipeline.
set -o pipefail
mkdir -p gpurun_out
for s in ${STREAMS:-1 2 3 2 1}; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --streams $s > gpurun_out/b_s$s.json 2> gpurun_out/b_s$s.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/b_s$s.json'));print('streams $s',d['value'],d['ms_per_step'],d['detail']['forward_ms_events'])"
done
