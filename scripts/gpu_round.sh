#!/bin/bash
# One GPU session: tests, bench, rocprofv3 kernel-trace summary (one batch in flight, so kernel
# durations are not stretched by a concurrent batch and agree with bench.py's serial per-op events).  Every GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; exit 1; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -m pytest tests -q -m gpu -s -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
  echo "gpu tests rc=$?"
fi
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --streams 1 > $OUT/prof.log 2>&1 || { echo rocprof failed; exit 1; }
echo done
