#!/bin/bash
set -e
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 scripts/detbench.hip -I yolo-series_amd/csrc -L yolo-series_amd/yv7 -lyv7 -Wl,-rpath,$PWD/yolo-series_amd/yv7 -o gpurun_out/detbench
timeout -k 10 120 gpurun_out/detbench 0,90,91,93,94,92,97 > gpurun_out/detbench.txt 2>&1
