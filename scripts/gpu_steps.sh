#!/bin/bash
# One GPU call as a chain of steps (the round's A/B drivers), each under its own time limit; the chain
# stops at the first failing step.  Outputs land in gpurun_out/TAG/.
#
# usage: bash scripts/gpu_steps.sh TAG STEP [STEP ...]
#   tests[=PYTEST_PATHS]        GPU suite (default: tests), -x, per-test timeout       -> tests.log
#   smoke                       __graft_entry__.smoke()                                -> smoke.log
#   ops[=NAME][@ENV=V,ENV=V]    serial per-op profile (scripts/op_profile.py) under the env; OPS_ARGS adds
#                               arguments (e.g. OPS_ARGS="--b 64")                    -> ops_NAME.txt
#   tune=OPS:CANDS[:ROUNDS]     tune_ops.py: each candidate forced on one op at a time -> tune.txt
#                               (OPS = all for every conv op)
#   bench[=N][@ENV=V,...]       N bench lines (default 2), --steps 40 --warmup 5  -> bench_STEP_I.json
#   benchw6[=N][@ENV=V,...]     the same for yolov7-w6 1280 bs 8                  -> benchw6_STEP_I.json
#   dispatch[=NAME]             scripts/dump_dispatch.py (default dispatch of the 3 bench plans) -> dispatch_NAME.txt
#   bench/benchw6 take BENCH_ARGS (extra bench.py arguments) from the environment
#   lib=NAME                    run the following steps on yolo-series_amd/yv7/libyv7_NAME.so (an
#                               A/B baseline built elsewhere); lib=cur restores the tree's library
# (round 5's one-shot launchers scripts/gpu_r5*.sh were folded into this driver, gpu_final.sh and
# gpu_prof.sh; they remain in the git history with the profiles they produced)
# e.g. bash scripts/gpu_steps.sh r4a tests ops=base ops=nodual@YV7_DUAL=0 tune=8,12:239,234:3 bench=2
#      bash scripts/gpu_steps.sh r4b ops=new lib=base ops=old lib=cur bench=1 lib=base bench=1 lib=cur
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=gpurun_out/$TAG
cd $R && mkdir -p $O
export PYTHONPATH=$R/yolo-series_amd:$R

envof() {   # "A=1,B=2" -> "A=1 B=2"
  [ -n "$1" ] && echo "${1//,/ }"
}

LIBD=$R/yolo-series_amd/yv7
n=0
for step in "$@"; do
  n=$((n + 1))
  name=${step%%=*}; arg=; [ "$step" != "$name" ] && arg=${step#*=}
  envs=; case "$arg" in *@*) envs=${arg#*@}; arg=${arg%%@*};; esac
  case "$name" in *@*) envs=${name#*@}; name=${name%%@*};; esac
  echo "== $step"
  case "$name" in
    tests)
      [ -z "$arg" ] && arg=tests
      timeout -k 10 600 python -u -m pytest ${arg//,/ } -m gpu -x -v --timeout 300 --timeout-method thread -rf \
        > $O/tests.log 2>&1
      rc=$?; grep -E "passed|failed" $O/tests.log | tail -1; grep -E "^FAILED" $O/tests.log | head
      [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
        || { cat $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    ops)
      f=$O/ops_${arg:-base}.txt
      env $(envof "$envs") timeout -k 10 300 python -u scripts/op_profile.py --top 100 $OPS_ARGS > $f 2>&1 || { tail $f; exit 1; }
      grep -E "^forward" $f ;;
    tune)
      IFS=: read -r ops cands rounds <<< "$arg"
      sel="--ops $ops"; [ "$ops" = all ] && sel=
      timeout -k 10 1100 python -u scripts/tune_ops.py $sel --cands $cands --rounds ${rounds:-2} $TUNE_ARGS \
        > $O/tune.txt 2>&1 || { tail -20 $O/tune.txt; exit 1; }
      grep -v amdgpu.ids $O/tune.txt | tail -90 ;;
    bench)
      for r in $(seq 1 ${arg:-2}); do
        f=$O/bench_${n}_$r.json
        env $(envof "$envs") timeout -k 10 300 python -u bench.py  --steps 40 --warmup 5 --no-cpu-baseline $BENCH_ARGS \
          > $f 2> ${f%.json}.err || exit 1
        python -c "import json;d=json.load(open('$f'));print('bench', '$f', '$envs', d['value'], d['detail']['serial_forward_ms'])"
      done ;;
    benchw6)
      for r in $(seq 1 ${arg:-2}); do
        f=$O/benchw6_${n}_$r.json
        env $(envof "$envs") timeout -k 10 300 python -u bench.py --model yolov7-w6 --batch 8 --img 1280 --steps 40 \
          --warmup 5 --no-cpu-baseline > $f 2> ${f%.json}.err || exit 1
        python -c "import json;d=json.load(open('$f'));print('benchw6', '$f', '$envs', d['value'], d['detail']['serial_forward_ms'])"
      done ;;
    dispatch)
      timeout -k 10 300 python -u scripts/dump_dispatch.py $O/dispatch_${arg:-cur}.txt > $O/dispatch_${arg:-cur}.log 2>&1 \
        || { tail $O/dispatch_${arg:-cur}.log; exit 1; }
      tail -1 $O/dispatch_${arg:-cur}.log ;;
    lib)
      [ -f $LIBD/libyv7_cur.so ] || cp $LIBD/libyv7.so $LIBD/libyv7_cur.so
      cp $LIBD/libyv7_$arg.so $LIBD/libyv7.so || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
