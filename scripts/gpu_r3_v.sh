#!/bin/bash
# Round 3 (v): GPU suite + smoke on the current tree, the profile pipeline (bench line, serial / bench
# kernel traces, per-kernel PMC traffic, roofline cross-check), then the batches-in-flight sweep.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r3v
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf > gpurun_out/r3v/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r3v/tests.log | tail -2; grep -E "^FAILED" gpurun_out/r3v/tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3v/smoke.log 2>&1 || { cat gpurun_out/r3v/smoke.log; exit 1; }
tail -1 gpurun_out/r3v/smoke.log
bash scripts/gpu_r3_prof.sh r3 70d01c0 || exit 1
for s in 2 4; do
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --streams $s > gpurun_out/r3v/bench_s$s.json 2> gpurun_out/r3v/bench_s$s.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r3v/bench_s$s.json'));print('streams $s', d['value'])"
done
