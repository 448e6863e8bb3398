#!/bin/bash
# Round 3 (b): GPU suite (new margin / w6 / fp8 config tests), the dispatch's kernel names, PMC passes
# of the 3x3 128->128 @80 kernels (default dispatch vs the halo ring).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r3
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread -rf > gpurun_out/r3/b_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r3/b_tests.log | tail -3; grep -E "^FAILED|Error" gpurun_out/r3/b_tests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "
import torch
from models.yolo import Model
from yv7.runtime import Plan
from yv7.synthetic import synthetic_state_dict
m = Model('yolov7'); synthetic_state_dict(m, seed=0); m = m.float().fuse().eval()
plan = Plan.from_model(m, 'cuda:0', torch.float16)
for i, k in enumerate(plan.op_kernels(32, 640, 640)): print(i, plan.graph.ops[i]['kind'], k)
" > gpurun_out/r3/op_kernels.txt 2>&1 || { tail -5 gpurun_out/r3/op_kernels.txt; exit 1; }
head -5 gpurun_out/r3/op_kernels.txt
bash scripts/pmc_cb.sh "3x3 128->128 @80" gpurun_out/r3/pmc_128 0 260
