#!/bin/bash
# Round 3 (z): GPU suite + smoke, serial per-op profile, bench line (twice) on the current tree.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3z}
O=gpurun_out/$TAG
cd $R && mkdir -p $O
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -2; grep -E "^FAILED" $O/tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u scripts/op_profile.py --top 100 > $O/ops.txt 2>&1 || exit 1
head -3 $O/ops.txt | tail -2
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_$r.json 2> $O/bench_$r.err || exit 1
  python -c "import json;d=json.load(open('$O/bench_$r.json'));print('round $r', d['value'], d['detail']['serial_forward_ms'])"
done
