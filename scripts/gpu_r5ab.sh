#!/bin/bash
# chunk-major K walk + XCD order in the 8-phase rings: tests, per-op PMC (yolov7, w6), A/B vs HEAD's library
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
bash scripts/gpu_steps.sh r5ab tests=tests/test_variants.py,tests/test_bench_config.py || exit 1
bash scripts/gpu_pmc_ops.sh r5ab/pmc_v7 || exit 1
bash scripts/gpu_pmc_ops.sh r5ab/pmc_w6 --model yolov7-w6 --b 8 --img 1280 || exit 1
bash scripts/gpu_steps.sh r5ab ops=new bench=2 benchw6=1 lib=base ops=old bench=2 benchw6=1 lib=cur bench=1 benchw6=1
