#!/bin/bash
# A/B of one dispatch environment knob on the default bench (3 batches in flight), interleaved
# runs in one box: usage  bash scripts/gpu_ab_env.sh NAME VAR VALUE_A VALUE_B [ROUNDS]
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
NAME=$1; VAR=$2; A=$3; B=$4; N=${5:-2}
for i in $(seq 1 $N); do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/${NAME}_${v}_$i.json 2> gpurun_out/${NAME}_${v}_$i.err || { tail gpurun_out/${NAME}_${v}_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['detail']['serial_forward_ms'])" gpurun_out/${NAME}_${v}_$i.json "$VAR=$v run $i"
  done
done
