#!/bin/bash
# HBM traffic of the bench workload from PMC counters: FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 passes (they do not fit one pass on gfx950), kernel-trace only, no other tracing.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o run -- \
    python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline --streams 1 > $OUT/pmc_$c.log 2>&1 || { echo "$c pass failed"; exit 1; }
done
echo done
