#!/bin/bash
set -e
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 scripts/convbench.hip -I yolo-series_amd/csrc -L yolo-series_amd/yv7 -lyv7 -Wl,-rpath,$PWD/yolo-series_amd/yv7 -o gpurun_out/convbench
CB_SHAPE="1x1" timeout -k 10 300 gpurun_out/convbench 0 201 296 297 298 > gpurun_out/cb1.txt 2>&1
