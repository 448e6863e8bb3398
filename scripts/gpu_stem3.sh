#!/bin/bash
# stem2 (restructured fused stem): hooks microbenchmark for both forms, the parity tests that reach
# the stem (bench config bs 32 op by op, fp16 layerwise), then a bench A/B of YV7_STEM 1 vs 2.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export PYTHONPATH=$R/yolo-series_amd:$R
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 scripts/stembench.hip -I yolo-series_amd/csrc -L yolo-series_amd/yv7 -lyv7 -Wl,-rpath,$PWD/yolo-series_amd/yv7 -o gpurun_out/stembench || exit 1
for f in 1 2; do for v in 0 1 2 3 4 0; do
  echo -n "form $f " >> gpurun_out/stem3.txt
  YV7_STEM=$f timeout -k 10 60 gpurun_out/stembench $v >> gpurun_out/stem3.txt 2>&1 || exit 1
done; done
cat gpurun_out/stem3.txt
timeout -k 10 600 python -u -m pytest tests/test_bench_config.py tests/test_gpu_forward.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/stem3_tests.log 2>&1 || { tail -40 gpurun_out/stem3_tests.log; exit 1; }
tail -2 gpurun_out/stem3_tests.log
bash scripts/gpu_ab_env.sh stem YV7_STEM 1 2 2
