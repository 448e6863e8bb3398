#!/bin/bash
# The BASELINE configs' bench lines on the current tree, one box: [1] yolov7 640 bs32 f16 (twice),
# [3] yolov7-w6 1280 bs8 f16, [4] yolov7 640 bs32 fp8 1x1, and yolov7-tiny 640 bs32.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r4lines}
O=gpurun_out/$TAG
cd $R && mkdir -p $O
export PYTHONPATH=$R/yolo-series_amd:$R
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n', d['value'], d['unit'], d['config'].get('workload'))"
}
run f16 && run w6 --model yolov7-w6 --img 1280 --batch 8 && run fp8 --dtype fp8 && run tiny --model yolov7-tiny && run f16b
# batches in flight on the current kernels (round 4): 2 and 4 streams beside the default 3
[ -n "$STREAMS_AB" ] && run s2 --streams 2 && run s4 --streams 4
true
