#!/bin/bash
# bench configuration probe on the current tree: batches in flight, HIP graph replay
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5j; mkdir -p $O; cd $R
export PYTHONPATH=$R/yolo-series_amd:$R
for args in "--streams 3" "--streams 2" "--streams 4" "--streams 3 --graph" "--streams 3"; do
  tag=$(echo $args | tr -d ' -')
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --no-cpu-baseline $args > $O/b_$tag.json 2> $O/b_$tag.err || exit 1
  python -c "import json;d=json.load(open('$O/b_$tag.json'));print('$args', d['value'], d['ms_per_step'])"
done
