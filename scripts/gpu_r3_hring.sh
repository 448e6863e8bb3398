#!/bin/bash
# Round 3: halo-ring 3x3 kernel (variants 260 / 261): per-op parity on every applicable layer, then the
# single-layer timing sweep on yolov7 bs32 640; then the round's baseline (GPU suite, bench, op profile).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r3
export PYTHONPATH=$R/yolo-series_amd:$R
for v in 260 261; do
  timeout -k 10 240 python -u scripts/check_variant.py $v yolov7 2 256 256 >> gpurun_out/r3/hring_check.log 2>&1 || { echo "check $v 256 failed"; tail -20 gpurun_out/r3/hring_check.log; exit 1; }
  timeout -k 10 240 python -u scripts/check_variant.py $v yolov7 2 640 640 >> gpurun_out/r3/hring_check.log 2>&1 || { echo "check $v 640 failed"; tail -20 gpurun_out/r3/hring_check.log; exit 1; }
done
cat gpurun_out/r3/hring_check.log | grep variant
timeout -k 10 300 python -u scripts/tune_ops.py --ops 13,14,15,16,83 --cands 260,261 --rounds 3 > gpurun_out/r3/hring_tune.txt 2>&1 || exit $?
cat gpurun_out/r3/hring_tune.txt | grep -v amdgpu.ids
bash scripts/gpu_r3_base.sh
