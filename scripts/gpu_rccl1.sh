#!/bin/bash
# RCCL data path on one GPU: the world-1 collective test, then the bench's multi-rank path under
# torch.distributed.run with one rank (YV7_BENCH_DIST=1: broadcast + per-batch all-gather issued).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 300 python -u -m pytest tests/test_dist.py tests/test_gpu_model_paths.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/rccl1_tests.log 2>&1 || { tail -40 gpurun_out/rccl1_tests.log; exit 1; }
tail -2 gpurun_out/rccl1_tests.log
YV7_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --no-cpu-baseline > gpurun_out/rccl1_bench.json 2> gpurun_out/rccl1_bench.err || { tail -30 gpurun_out/rccl1_bench.err; exit 1; }
cat gpurun_out/rccl1_bench.json
