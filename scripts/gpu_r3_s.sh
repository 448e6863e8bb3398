#!/bin/bash
# Round 3 (s): register-streamed 1x1 (conv_rs.hip): forced variant 240 and the runtime's dual launch of
# the MP block's two readers; GPU suite, single-layer sweep, bench A/B against YV7_DUAL=0.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3s}
O=gpurun_out/$TAG
cd $R && mkdir -p $O
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 300 python -u -m pytest tests/test_variants.py tests/test_bench_config.py -m gpu -x -v --timeout 240 --timeout-method thread -rf > $O/tests_a.log 2>&1
rc=$?; echo "pytest(a) rc=$rc"; grep -E "passed|failed" $O/tests_a.log | tail -2; grep -E "^FAILED|Error|error" $O/tests_a.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/tune_ops.py --ops 3,8,9,10,12,59,64,65,66 --cands 240 --rounds 3 > $O/tune.txt 2>&1 || { tail -20 $O/tune.txt; exit 1; }
grep -v amdgpu.ids $O/tune.txt
for r in 1 2; do
  YV7_DUAL=0 timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_old_$r.json 2> $O/bench_old_$r.err || exit 1
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bench_new_$r.json 2> $O/bench_new_$r.err || exit 1
  for v in old new; do python -c "import json;d=json.load(open('$O/bench_${v}_$r.json'));print('$v round $r', d['value'], d['detail']['serial_forward_ms'])"; done
done
timeout -k 10 300 python -u scripts/op_profile.py --top 100 > $O/ops.txt 2>&1 || exit 1
YV7_DUAL=0 timeout -k 10 300 python -u scripts/op_profile.py --top 100 > $O/ops_nodual.txt 2>&1 || exit 1
grep -E '^ *(3|8|9|10|12|59|64|65|66) ' $O/ops.txt $O/ops_nodual.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -2; grep -E "^FAILED" $O/tests.log | head
