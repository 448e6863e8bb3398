#!/bin/bash
# The multi-rank bench path on ONE MI355X: torch.distributed.run with one rank, YV7_BENCH_DIST=1 forcing the
# RCCL weight broadcast, the per-batch detection all-gather, the process-group timeout and the progress
# watchdog (yv7/dist.py) that the driver's N > 1 runs use.
# usage: bash scripts/gpu_rccl1.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-rccl1}
mkdir -p $O && cd $R
YV7_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_rccl1.json 2> $O/bench_rccl1.err || exit $?
[ $(wc -l < $O/bench_rccl1.json) -eq 1 ] || { echo "stdout is not one JSON line"; exit 1; }
python -c "import json;d=json.load(open('$O/bench_rccl1.json'));print('rccl world 1', d['value'], d['config']['rccl_world_size'], d['detail'].get('allgather_us_per_batch'))"
