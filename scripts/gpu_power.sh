#!/bin/bash
# Power / clock trace of a long bench run (is the chip power-limited under the batches in flight?):
# rocm-smi sampled every ~0.5 s beside `bench.py --steps 1500`, plus an idle sample before.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3pw}; shift; EXTRA="$@"   # extra bench.py arguments, e.g. --streams 1
O=gpurun_out/$TAG
cd $R && mkdir -p $O
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 5 20 rocm-smi --showpower --showclocks --showtemp > $O/idle.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 1500 --warmup 20 --no-cpu-baseline $EXTRA > $O/bench.json 2> $O/bench.err &
BP=$!
for i in $(seq 1 60); do
  kill -0 $BP 2>/dev/null || break
  echo "== t=$i" >> $O/smi.txt
  timeout -k 5 10 rocm-smi --showpower --showclocks --showtemp >> $O/smi.txt 2>&1
  sleep 0.5
done
wait $BP; rc=$?
echo "bench rc=$rc"; cat $O/bench.json | python -c "import json,sys;d=json.load(sys.stdin);print(d['value'],d['ms_per_step'])"
grep -iE "power|sclk|fclk|mclk|temperature \(Sensor junction" $O/smi.txt | sort | uniq -c | sort -rn | head -30
exit $rc
