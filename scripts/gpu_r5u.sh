#!/bin/bash
# batches in flight vs the power cap: bench at 1-4 streams, then rocm-smi power traces at 1 and 3
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5u; mkdir -p $O; cd $R
export PYTHONPATH=$R/yolo-series_amd:$R
for s in 1 2 3 4 3 1; do
  timeout -k 10 200 python -u bench.py --steps 60 --warmup 5 --no-cpu-baseline --streams $s > $O/bench_s$s.json 2> $O/bench_s$s.err || exit 1
  python -c "import json;d=json.load(open('$O/bench_s$s.json'));print('streams $s',d['value'],d['ms_per_step'])"
done
bash scripts/gpu_power.sh r5u/pw3 && bash scripts/gpu_power.sh r5u/pw1 --streams 1 || exit 1
# per-image op times at small batches (front tensors MALL-resident between ops) vs bs 32
for b in 4 8 32; do
  timeout -k 10 200 python -u scripts/op_profile.py --b $b --top 100 > $O/ops_b$b.txt 2>&1 || exit 1
  grep -E "^forward" $O/ops_b$b.txt
done
