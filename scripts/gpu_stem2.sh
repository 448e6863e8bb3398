#!/bin/bash
set -e
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 scripts/stembench.hip -I yolo-series_amd/csrc -L yolo-series_amd/yv7 -lyv7 -Wl,-rpath,$PWD/yolo-series_amd/yv7 -o gpurun_out/stembench
for v in 0 1 2 3 4 0; do timeout -k 10 60 gpurun_out/stembench $v >> gpurun_out/stem2.txt 2>&1; done
