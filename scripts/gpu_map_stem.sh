#!/bin/bash
# mAP@0.5 parity of the bench frames against the fp32 oracle with the first-form stem vs stem2.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for f in 2; do
  YV7_STEM=$f timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-seconds 2 > gpurun_out/mapstem_$f.json 2> gpurun_out/mapstem_$f.err || { tail gpurun_out/mapstem_$f.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d.get('map50_parity'), d['cpu_baseline']['map_parity'])" gpurun_out/mapstem_$f.json
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 scripts/stembench.hip -I yolo-series_amd/csrc -L yolo-series_amd/yv7 -lyv7 -Wl,-rpath,$PWD/yolo-series_amd/yv7 -o gpurun_out/stembench || exit 1
for f in 1 2 2; do echo -n "form $f "; YV7_STEM=$f timeout -k 10 60 gpurun_out/stembench 0 || exit 1; done
