#!/bin/bash
# Round 3 (h): same-box A/B of the halo ring in the dispatch (YV7_HRING=0 vs default, interleaved),
# and the library-GEMM reference point for the layer shapes.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3h}
cd $R && mkdir -p gpurun_out/$TAG
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 180 python -u scripts/gemm_ref.py > gpurun_out/$TAG/gemm_ref.txt 2>&1 || { cat gpurun_out/$TAG/gemm_ref.txt; exit 1; }
cat gpurun_out/$TAG/gemm_ref.txt
for r in 1 2; do
  for h in 1 0; do
    YV7_HRING=$h timeout -k 10 240 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/$TAG/bench_h${h}_$r.json 2> gpurun_out/$TAG/bench_h${h}_$r.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/$TAG/bench_h${h}_$r.json'));print('HRING=$h round $r', d['value'], d['detail']['serial_forward_ms'])"
  done
done
