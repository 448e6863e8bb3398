#!/bin/bash
# Round 3 (p): ws64 half-patch ring (variant 15, default) vs the column-pair form (11): microbench with
# hooks (114/116 ring, 14/16 pair), same-box A/B against the previous library, GPU suite, bench A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3p}
O=gpurun_out/$TAG
cd $R && mkdir -p $O
export PYTHONPATH=$R/yolo-series_amd:$R
CB_SHAPE="3x3 64->64 @" timeout -k 10 120 scripts/convbench 0 11 114 116 14 16 0 11 > $O/cb_new.txt 2>&1 || { cat $O/cb_new.txt; exit 1; }
cat $O/cb_new.txt
CB_SHAPE="3x3 64->64 @" timeout -k 10 120 ab/convbench_old 0 > $O/cb_old.txt 2>&1 || { cat $O/cb_old.txt; exit 1; }
cat $O/cb_old.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -2; grep -E "^FAILED" $O/tests.log | head
[ $rc -eq 0 ] || exit $rc
rm -rf /tmp/oldtree && mkdir -p /tmp/oldtree && cp -r $R/. /tmp/oldtree/ && cp ab/libyv7.so /tmp/oldtree/yolo-series_amd/yv7/libyv7.so
for r in 1 2; do
  (cd /tmp/oldtree && PYTHONPATH=/tmp/oldtree/yolo-series_amd:/tmp/oldtree timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > $R/$O/bench_old_$r.json 2> $R/$O/bench_old_$r.err) || exit 1
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_new_$r.json 2> $O/bench_new_$r.err || exit 1
  for v in old new; do python -c "import json;d=json.load(open('$O/bench_${v}_$r.json'));print('$v round $r', d['value'], d['detail']['serial_forward_ms'])"; done
done
timeout -k 10 300 python -u scripts/op_profile.py --top 100 > $O/ops.txt 2>&1 || exit 1
head -12 $O/ops.txt
