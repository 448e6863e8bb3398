#!/bin/bash
# Round 3 (r): sibling 1x1 convs with outputs in separate tensors fused into one GEMM (graph pass
# _merge_sibling_tensors): GPU suite, per-layer candidates on the three merged ops, bench A/B against
# YV7_NO_TMERGE=1 (same library).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3r}
O=gpurun_out/$TAG
cd $R && mkdir -p $O
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -2; grep -E "^FAILED" $O/tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/tune_ops.py --ops 19,29,37 --cands 201,202,204,205,206,231,232 --rounds 3 > $O/tune.txt 2>&1 || { tail -20 $O/tune.txt; exit 1; }
grep -v amdgpu.ids $O/tune.txt
for r in 1 2; do
  YV7_NO_TMERGE=1 timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_old_$r.json 2> $O/bench_old_$r.err || exit 1
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_new_$r.json 2> $O/bench_new_$r.err || exit 1
  for v in old new; do python -c "import json;d=json.load(open('$O/bench_${v}_$r.json'));print('$v round $r', d['value'], d['detail']['serial_forward_ms'])"; done
done
timeout -k 10 300 python -u scripts/op_profile.py --top 100 > $O/ops.txt 2>&1 || exit 1
grep -E '^ *(19|29|37) ' $O/ops.txt
