#!/bin/bash
# Round 3 (x): persistent Detect head with tile t's sigmoid staging pipelined into tile t + 1's first K
# step — same-box A/B against the previous library (ab/), GPU suite, bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3x}
O=gpurun_out/$TAG
cd $R && mkdir -p $O
export PYTHONPATH=$R/yolo-series_amd:$R
for r in 1 2; do
  timeout -k 10 180 ab/detbench_old 0 > $O/det_old_$r.txt 2>&1 || { cat $O/det_old_$r.txt; exit 1; }
  timeout -k 10 180 scripts/detbench 0,98 > $O/det_new_$r.txt 2>&1 || { cat $O/det_new_$r.txt; exit 1; }
done
for f in $O/det_*.txt; do echo "== $f"; cat $f; done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -2; grep -E "^FAILED" $O/tests.log | head
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_$r.json 2> $O/bench_$r.err || exit 1
  python -c "import json;d=json.load(open('$O/bench_$r.json'));print('round $r', d['value'], d['detail']['serial_forward_ms'])"
done
