#!/bin/bash
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD/yolo-series_amd:$PWD
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 scripts/detbench.hip -I yolo-series_amd/csrc -L yolo-series_amd/yv7 -lyv7 -Wl,-rpath,$PWD/yolo-series_amd/yv7 -o gpurun_out/detbench
timeout -k 10 120 gpurun_out/detbench 0,90,91,93,94 > gpurun_out/nt_detbench.txt 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_nms.py tests/test_bench_config.py > gpurun_out/nt_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 60 --no-cpu-baseline > gpurun_out/nt_bench_$i.json 2> gpurun_out/nt_bench_$i.err
done
