#!/bin/bash
# Round 3 (o): ws64 with its epilogue interleaved into the MFMA stream (compile-time hooks) and the next
# tile's first weight set prefetched — same-box A/B against the previous library (ab/libyv7.so), the
# GPU suite, then the bench line old/new alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3o}
O=gpurun_out/$TAG
cd $R && mkdir -p $O
export PYTHONPATH=$R/yolo-series_amd:$R
for r in 1 2; do
  CB_SHAPE="3x3 64->64 @" timeout -k 10 120 ab/convbench_old 0 14 16 > $O/cb_old_$r.txt 2>&1 || { cat $O/cb_old_$r.txt; exit 1; }
  CB_SHAPE="3x3 64->64 @" timeout -k 10 120 scripts/convbench 0 14 16 > $O/cb_new_$r.txt 2>&1 || { cat $O/cb_new_$r.txt; exit 1; }
done
for f in $O/cb_*.txt; do echo "== $f"; cat $f; done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -2; grep -E "^FAILED" $O/tests.log | head
[ $rc -eq 0 ] || exit $rc
rm -rf /tmp/oldtree && mkdir -p /tmp/oldtree && cp -r $R/. /tmp/oldtree/ && cp ab/libyv7.so /tmp/oldtree/yolo-series_amd/yv7/libyv7.so
for r in 1 2; do
  (cd /tmp/oldtree && PYTHONPATH=/tmp/oldtree/yolo-series_amd:/tmp/oldtree timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > $R/$O/bench_old_$r.json 2> $R/$O/bench_old_$r.err) || exit 1
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_new_$r.json 2> $O/bench_new_$r.err || exit 1
  for v in old new; do python -c "import json;d=json.load(open('$O/bench_${v}_$r.json'));print('$v round $r', d['value'], d['detail']['serial_forward_ms'])"; done
done
