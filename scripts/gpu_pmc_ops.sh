#!/bin/bash
# Per-op HBM traffic of the serial bench plan (yolov7 640 bs32 f16 unless OP_ARGS says otherwise):
# op_profile.py --dump, then FETCH_SIZE and WRITE_SIZE in separate --pmc passes, then scripts/pmc_ops.py.
# usage: bash scripts/gpu_pmc_ops.sh TAG [op_profile args...]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
export PYTHONPATH=$R/yolo-series_amd:$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/scripts/op_profile.py --iters 3 --top 100 --dump $O/ops.json "$@" > $O/ops.txt 2>&1 || { tail $O/ops.txt; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$c -o run -- python3 $R/scripts/op_profile.py --iters 1 "$@" > $O/pmc_$c.log 2>&1 || { echo "$c pass failed"; exit 1; }
done
cd $R && python3 scripts/pmc_ops.py $O/ops.json $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE $O/pmc_ops.txt > /dev/null && tail -3 $O/pmc_ops.txt
