#!/bin/bash
# stem forms 2 (two blocks per CU, phases across barriers) vs 3 (software-pipelined, one block per
# CU): hook microbenchmark, parity tests under form 3, bench A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export PYTHONPATH=$R/yolo-series_amd:$R
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 scripts/stembench.hip -I yolo-series_amd/csrc -L yolo-series_amd/yv7 -lyv7 -Wl,-rpath,$PWD/yolo-series_amd/yv7 -o gpurun_out/stembench || exit 1
for f in 2 3; do for v in 0 3 0; do
  echo -n "form $f " >> gpurun_out/stem4.txt
  YV7_STEM=$f timeout -k 10 60 gpurun_out/stembench $v >> gpurun_out/stem4.txt 2>&1 || exit 1
done; done
cat gpurun_out/stem4.txt
YV7_STEM=3 timeout -k 10 600 python -u -m pytest tests/test_bench_config.py tests/test_gpu_forward.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/stem4_tests.log 2>&1 || { tail -40 gpurun_out/stem4_tests.log; exit 1; }
tail -2 gpurun_out/stem4_tests.log
bash scripts/gpu_ab_env.sh stem4 YV7_STEM 2 3 2
