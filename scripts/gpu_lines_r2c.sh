#!/bin/bash
# Bench lines of the other BASELINE configs after the stem2 change, and a streams re-check.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
run() { n=$1; shift; timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/l_$n.json 2> gpurun_out/l_$n.err || { tail gpurun_out/l_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['detail']['serial_forward_ms'])" gpurun_out/l_$n.json; }
run f16 && run fp8 --dtype fp8 && run f16_s4 --streams 4 && run f16_s2 --streams 2 && run w6 --model yolov7-w6 --img 1280 --batch 8 && run tiny --model yolov7-tiny && run f16b
