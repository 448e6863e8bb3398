#!/bin/bash
# A/B: HIP stream priorities of the batches in flight (bench --prio).
set -o pipefail
mkdir -p gpurun_out
for pr in "" "-1,0,0" "-1,-1,0" "" "-1,0,0"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 ${pr:+--prio=$pr} > gpurun_out/b_prio.json 2> gpurun_out/b_prio.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/b_prio.json'));print('prio [$pr]',d['value'],d['ms_per_step'])"
done
