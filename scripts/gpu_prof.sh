#!/bin/bash
# Per-round profiles of the CURRENT tree (bench config yolov7 640 bs32 f16): the rocprofv3 kernel trace of
# serial forwards (the roofline's per-kernel launch times), the per-kernel HBM traffic (FETCH_SIZE /
# WRITE_SIZE in separate --pmc passes), then the default bench line and its own kernel trace.
# usage: bash scripts/gpu_prof.sh TAG TREE   (TAG r4 writes profiles/r4_pmc_traffic.json, which bench.py reads)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r4}; TREE=${2:-}
O=gpurun_out/$TAG
cd $R && mkdir -p $O
export PYTHONPATH=$R/yolo-series_amd:$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/serial_kt -o kt -- python3 $R/scripts/op_profile.py --top 100 --dump $R/$O/serial_ops.json > $R/$O/serial_ops.txt 2> $R/$O/serial_kt.err || { echo "serial trace failed"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $R/$O/pmc_$c -o run -- python3 $R/scripts/op_profile.py --iters 3 > $R/$O/pmc_$c.log 2>&1 || { echo "$c pass failed"; exit 1; }
done
cd $R && python3 scripts/pmc_traffic_kernels.py $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE $O/pmc_traffic.json "$TREE" || exit 1
cp $O/pmc_traffic.json profiles/${TAG}_pmc_traffic.json
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/bench_kt -o kt -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/$O/bench_kt.json 2> $R/$O/bench_kt.err || exit 1
cd $R && python3 scripts/roofline_check.py $O/serial_kt $O/bench.json $O/serial_ops.json > $O/roofline_check.txt; cat $O/roofline_check.txt
