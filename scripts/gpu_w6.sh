#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-w6}; mkdir -p $O; cd $R
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 300 python -u scripts/op_profile.py --model yolov7-w6 --b 8 --img 1280 --top 120 > $O/ops_w6.txt 2>&1 || { tail $O/ops_w6.txt; exit 1; }
head -3 $O/ops_w6.txt | tail -1; grep "k3 s2" $O/ops_w6.txt; tail -9 $O/ops_w6.txt
timeout -k 10 300 python -u bench.py --model yolov7-w6 --batch 8 --img 1280 --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_w6.json 2> $O/bench_w6.err || exit 1
python -c "import json;d=json.load(open('$O/bench_w6.json'));print('w6 bench', d['value'], d['roofline']['job_frac'], d['detail']['serial_forward_ms'])"
