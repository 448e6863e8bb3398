#!/bin/bash
# w6 1280 bs8: batches in flight 2 / 3 / 4 / 5
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5w6s; mkdir -p $O; cd $R
export PYTHONPATH=$R/yolo-series_amd:$R
for s in 3 2 4 5 3; do
  timeout -k 10 200 python -u bench.py --model yolov7-w6 --batch 8 --img 1280 --steps 60 --warmup 5 --no-cpu-baseline --streams $s > $O/w6_s$s.json 2> $O/w6_s$s.err || exit 1
  python -c "import json;d=json.load(open('$O/w6_s$s.json'));print('w6 streams $s',d['value'],d['ms_per_step'])"
done
